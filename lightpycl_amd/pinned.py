"""Page-locked host blocks for the results export (lpc_host_alloc / lpc_host_free).

The drop-in's results mode hands the caller numpy arrays (the reference's
per-iteration results tuples, iterative_tracer.py:335-355).  They live in
page-locked, device-mapped memory so that the copy of an iteration to the host
runs on the export stream beside the next iteration's kernels
(lpc_trace_iterate_export: a copy kernel writing the mapped block over PCIe,
since round 5; a DMA for a block the device cannot map).  Pinning pages costs
milliseconds per tens of MB,
so blocks are recycled: a block returns to the pool when the last numpy array
viewing it is garbage-collected (the arrays keep the block alive through their
``base``), and the next trace of a similar size reuses it.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from . import _lib


def _size_class(nbytes):
    """Round up to 2^k or 1.5 * 2^k bytes (at most a third wasted), >= 64 KiB."""
    n = max(int(nbytes), 1 << 16)
    k = n.bit_length() - 1
    if n == 1 << k:
        return n
    mid = (1 << k) + (1 << (k - 1))
    return mid if n <= mid else 1 << (k + 1)


class _Owner:
    """Returns its block to the pool when the last view is gone."""

    __slots__ = ("pool", "ptr", "size")

    def __init__(self, pool, ptr, size):
        self.pool, self.ptr, self.size = pool, ptr, size

    def __del__(self):
        try:
            self.pool._put(self.ptr, self.size)
        except Exception:
            pass


class PinnedPool:
    """Size-classed free lists of pinned blocks, at most ``keep_bytes`` idle."""

    def __init__(self, keep_bytes=8 << 30):
        self.keep_bytes = int(keep_bytes)
        self._free = {}
        self._idle = 0
        self._lock = threading.Lock()
        self.allocated = 0          # blocks pinned over the pool's life (diagnostics)

    def block(self, nbytes):
        """A ctypes char array over a pinned block of >= nbytes (its ``_owner``
        recycles the block once nothing references the array)."""
        size = _size_class(nbytes)
        with self._lock:
            lst = self._free.get(size)
            ptr = lst.pop() if lst else None
            if ptr is not None:
                self._idle -= size
        if ptr is None:
            # an empty size class: pin the block and, when it fits under keep_bytes,
            # a spare -- a caller that keeps the previous call's results alive (the
            # tracer's own .results, until its next call replaces them) needs two
            # sets in turn, and pinning on the next call would cost that call
            # milliseconds.  A spare that would not fit is
            # not pinned at all (it would be unpinned at once)
            L = _lib.load()
            with self._lock:
                spare = self._idle + size <= self.keep_bytes
            got = []
            for _ in range(2 if spare else 1):
                p = ctypes.c_void_p()
                _lib.check(L.lpc_host_alloc(size, ctypes.byref(p)), None)
                got.append(p.value)
                self.allocated += 1
            ptr = got[0]
            if spare:
                self._put(got[1], size)
        arr = (ctypes.c_char * size).from_address(ptr)
        arr._owner = _Owner(self, ptr, size)
        return arr

    def _put(self, ptr, size):
        with self._lock:
            if self._idle + size <= self.keep_bytes:
                self._free.setdefault(size, []).append(ptr)
                self._idle += size
                return
        _lib.load().lpc_host_free(ctypes.c_void_p(ptr))

    def views(self, blk, layout):
        """numpy views of consecutive sections of ``blk``: layout = [(dtype, shape)]."""
        out, off = [], 0
        for dt, shape in layout:
            cnt = int(np.prod(shape))
            a = np.frombuffer(blk, dtype=dt, count=cnt, offset=off).reshape(shape)
            out.append(a)
            off += cnt * np.dtype(dt).itemsize
        return out


POOL = PinnedPool()
