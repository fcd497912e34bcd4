"""dataplug_amd: MI355X-native record-boundary indexing for dataplug-style cloud objects.

The user surface mirrors CLOUDLAB-URV/dataplug (``CloudObject``, ``CloudDataFormat``, format plugins and
partition strategies); the byte scans that build the indexes run as hand-written HIP kernels on gfx950
(``dataplug_amd/csrc/dpscan.hip`` behind the C ABI in ``include/dpscan.h``).
"""
from .version import __version__  # noqa: F401


def __getattr__(name):
    # lazy: importing the package must not pull in pandas/joblib or load the HIP library
    if name == "CloudObject":
        from .cloudobject import CloudObject
        return CloudObject
    if name in ("CloudDataFormat", "CloudObjectSlice", "PartitioningStrategy", "PreprocessingType"):
        from . import entities
        return getattr(entities, name)
    if name == "PreprocessingMetadata":
        from .preprocessing.metadata import PreprocessingMetadata
        return PreprocessingMetadata
    raise AttributeError(name)
