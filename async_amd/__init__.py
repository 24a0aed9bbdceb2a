"""async_amd -- MI355X-native base64 byte-stream stage for the `async`
library's bytestream_1 interface.

The product is the C ABI in libasync_b64.so (include/*.h): the drop-in
bytestream_1 stages (base64_encode / base64_decode and their methods), the
device/batch entry points (b64x_*), and the minimal event loop and streams
they run on.  This package only locates and binds that library; see
``async_amd.b64`` for the device-tensor API used by tests and bench.py.
"""
from ._lib import LIB_PATH, B64xError, alphabet, load  # noqa: F401

__all__ = ["LIB_PATH", "B64xError", "alphabet", "load"]
