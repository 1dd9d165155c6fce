"""PMC calibration for 8-B-per-lane streams (run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE on
the GPU box): k_calib_read8 reads and k_calib_write8 writes N doubles, coalesced.  The counter
value per launch over 8*N bytes is the correction factor for the path kernels' access width."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lumo_amd as L  # noqa: E402
from lumo_amd import _ffi  # noqa: E402

N = 1 << 27  # 1 GiB: well past the 256 MiB Infinity Cache
dev = L.Device(0)
_ffi.check(_ffi.load().lumo_debug_stream(dev.ctx, N), "debug_stream")
dev.close()
print(f"calib: {8 * N} bytes read by k_calib_read8, {8 * N} bytes written by k_calib_write8")
