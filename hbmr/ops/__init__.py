"""Hand-written MI355X kernels exposed to the runtime (libhbmr.so via ctypes)."""
from . import _lib  # noqa: F401
from ._lib import NativeLibraryError, available, load  # noqa: F401
