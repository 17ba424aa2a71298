"""Device memory for tests that hand raw device buffers to the C ABI: a thin
ctypes view of the HIP runtime (hipMalloc / hipMemcpy / hipFree), so the
tests need no torch.  Test infrastructure only."""
import ctypes

import numpy as np

_hip = None


def hip():
    global _hip
    if _hip is None:
        h = ctypes.CDLL("libamdhip64.so")
        h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        h.hipFree.argtypes = [ctypes.c_void_p]
        h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        h.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
        h.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        h.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        h.hipStreamDestroy.argtypes = [ctypes.c_void_p]
        h.hipSetDevice.argtypes = [ctypes.c_int]
        _hip = h
    return _hip


def _ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


class DeviceBuffer:
    """n bytes of device memory on the current device."""

    def __init__(self, nbytes: int, fill: int | None = None):
        self.nbytes = max(int(nbytes), 1)
        self._p = ctypes.c_void_p()
        _ok(hip().hipMalloc(ctypes.byref(self._p), self.nbytes), "hipMalloc")
        if fill is not None:
            _ok(hip().hipMemset(self._p, fill, self.nbytes), "hipMemset")

    @property
    def ptr(self) -> int:
        return self._p.value

    def upload(self, data) -> "DeviceBuffer":
        a = np.frombuffer(bytes(data), dtype=np.uint8) if isinstance(data, (bytes, bytearray)) \
            else np.ascontiguousarray(data)
        if a.nbytes:
            assert a.nbytes <= self.nbytes
            _ok(hip().hipMemcpy(self._p, a.ctypes.data, a.nbytes, 1), "hipMemcpy H2D")
        return self

    def download(self, dtype, count: int | None = None) -> np.ndarray:
        dt = np.dtype(dtype)
        n = self.nbytes // dt.itemsize if count is None else count
        out = np.empty(n, dtype=dt)
        if out.nbytes:
            _ok(hip().hipMemcpy(out.ctypes.data, self._p, out.nbytes, 2), "hipMemcpy D2H")
        return out

    def close(self):
        if self._p:
            hip().hipFree(self._p)
            self._p = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def copy_from_device(ptr: int, dtype, count: int) -> np.ndarray:
    out = np.empty(count, dtype=np.dtype(dtype))
    if out.nbytes:
        _ok(hip().hipMemcpy(out.ctypes.data, ctypes.c_void_p(ptr), out.nbytes, 2), "hipMemcpy D2H")
    return out


class Stream:
    def __init__(self):
        self._s = ctypes.c_void_p()
        _ok(hip().hipStreamCreate(ctypes.byref(self._s)), "hipStreamCreate")

    @property
    def handle(self):
        return self._s

    def synchronize(self):
        _ok(hip().hipStreamSynchronize(self._s), "hipStreamSynchronize")

    def close(self):
        if self._s:
            hip().hipStreamDestroy(self._s)
            self._s = ctypes.c_void_p()


def device_synchronize():
    _ok(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
