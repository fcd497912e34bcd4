"""dataplug_amd — MI355X-native record-boundary indexing for dataplug's CloudObject / plugin API."""
from .version import __version__  # noqa: F401
