"""HIP record-boundary scans (libdpscan.so via ctypes).  No CPU fallback: see _lib.DPScanUnavailable."""
from ._lib import DPCapacityError, DPScanError, DPScanUnavailable, LIB_PATH, load  # noqa: F401
from .device import DeviceBuffer, ScanContext, device_count, get_context, pick_device  # noqa: F401
