"""Streaming writer for ray histories.

The reference's lightsheet sweep (scripts/2024_04_01_lightsheet.py:53-60, 134-135) stores one history
per configuration in a zarr array ``rays`` of shape (n_config, planes, n_rays, 8) chunked one
configuration per chunk, with ``array_columns`` = x, y, z, dx, dy, dz, phase, wavelength.  zarr is
not a dependency here, so :class:`HistoryWriter` writes that exact layout as a zarr-v2 directory store
itself (uncompressed chunks, ``.zarray`` / ``.zattrs`` / ``.zgroup`` JSON), readable by zarr when it is
installed and by :func:`read_array` otherwise.

Histories may be NumPy arrays or torch CUDA tensors.  Device histories are copied into pinned host
buffers on a side stream and written by a background thread, so the GPU can trace the next
configuration while the previous one goes to disk (double-buffered).
"""
import json
import os
import queue
import threading

import numpy as np

from . import _engine as E

ARRAY_COLUMNS = ["x", "y", "z", "dx", "dy", "dz", "phase", "wavelength"]


def _zarray(shape, chunks, dtype):
    return {"zarr_format": 2, "shape": list(shape), "chunks": list(chunks), "dtype": np.dtype(dtype).str,
            "compressor": None, "fill_value": "NaN" if np.dtype(dtype).kind == "f" else 0, "filters": None,
            "order": "C", "dimension_separator": "."}


def _write_json(path, obj):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f, indent=1)
    os.replace(tmp, path)


class HistoryWriter:
    """zarr-v2 store at ``path`` with array ``rays`` (n_configs, n_planes, n_rays, 8)."""

    def __init__(self, path, n_configs, n_planes, n_rays, dtype="float64", attrs=None, depth=2):
        self.path = str(path)
        self.shape = (int(n_configs), int(n_planes), int(n_rays), 8)
        self.dtype = np.dtype(dtype)
        os.makedirs(os.path.join(self.path, "rays"), exist_ok=True)
        _write_json(os.path.join(self.path, ".zgroup"), {"zarr_format": 2})
        _write_json(os.path.join(self.path, ".zattrs"), dict(attrs or {}))
        _write_json(os.path.join(self.path, "rays", ".zarray"), _zarray(self.shape, (1,) + self.shape[1:], self.dtype))
        _write_json(os.path.join(self.path, "rays", ".zattrs"), {"array_columns": ARRAY_COLUMNS})
        self._q = queue.Queue(maxsize=depth)
        self._free = queue.Queue()
        self._err = None
        self._pinned = []
        self._thread = threading.Thread(target=self._drain, daemon=True)
        self._thread.start()

    # -------------------------------------------------------------------- chunks
    def _chunk_file(self, index):
        return os.path.join(self.path, "rays", f"{index}.0.0.0")

    def _drain(self):
        while True:
            item = self._q.get()
            if item is None:
                return
            index, arr, event, buf, src = item
            item = None
            try:
                if event is not None:
                    event.synchronize()
                # the copy has finished: drop the last references to the device history, so its memory may be
                # freed (and reused by the next trace) while this chunk goes to disk
                del src
                tmp = self._chunk_file(index) + ".tmp"
                with open(tmp, "wb") as f:
                    f.write(memoryview(np.ascontiguousarray(arr)).cast("B"))
                os.replace(tmp, self._chunk_file(index))
            except Exception as e:  # surfaced by the next write()/close()
                self._err = e
            finally:
                if buf is not None:
                    self._free.put(buf)

    def write(self, index, history):
        """Store ``history`` (n_planes, n_rays, 8) as configuration ``index`` (asynchronous)."""
        if self._err is not None:
            raise self._err
        if not 0 <= index < self.shape[0]:
            raise IndexError(index)
        if tuple(history.shape) != self.shape[1:]:
            raise ValueError(f"history shape {tuple(history.shape)} != {self.shape[1:]}")
        t = type(history)
        if t.__module__.startswith("torch") and history.is_cuda:
            import torch
            try:
                buf = self._free.get_nowait()
            except queue.Empty:
                tdt = torch.float64 if self.dtype == np.float64 else torch.float32
                buf = torch.empty(self.shape[1:], dtype=tdt, pin_memory=True)
                self._pinned.append(buf)
            stream = torch.cuda.Stream(history.device)
            stream.wait_stream(torch.cuda.current_stream(history.device))
            with torch.cuda.stream(stream):
                buf.copy_(history, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(stream)
            # the copy reads `history` on the side stream: recorded (torch's allocator; E.record_stream also
            # covers a buffer of the library's own C-ABI pool), and the queue item holds the tensor until the
            # copy has finished, so its memory is not handed to the next trace while the copy is in flight
            E.record_stream(history, stream)
            self._q.put((index, buf.numpy(), ev, buf, history))
        else:
            self._q.put((index, np.asarray(history, dtype=self.dtype).copy(), None, None, None))

    def write_array(self, name, values):
        """A small companion array (e.g. the swept parameter), like ``z.array(name, values)``."""
        values = np.ascontiguousarray(values)
        os.makedirs(os.path.join(self.path, name), exist_ok=True)
        _write_json(os.path.join(self.path, name, ".zarray"), _zarray(values.shape, values.shape, values.dtype))
        with open(os.path.join(self.path, name, ".".join(["0"] * max(values.ndim, 1))), "wb") as f:
            f.write(values.tobytes())

    def close(self):
        self._q.put(None)
        self._thread.join()
        if self._err is not None:
            raise self._err

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_array(path, name="rays"):
    """Read an array written by HistoryWriter (unwritten chunks come back as NaN / fill)."""
    with open(os.path.join(path, name, ".zarray")) as f:
        meta = json.load(f)
    dtype = np.dtype(meta["dtype"])
    shape, chunks = tuple(meta["shape"]), tuple(meta["chunks"])
    fill = np.nan if meta["fill_value"] == "NaN" else meta["fill_value"]
    out = np.full(shape, fill, dtype=dtype)
    grid = [range(-(-s // c)) for s, c in zip(shape, chunks)]
    for idx in np.ndindex(*[len(g) for g in grid]):
        fn = os.path.join(path, name, ".".join(str(i) for i in idx) if idx else "0")
        if not os.path.exists(fn):
            continue
        block = np.fromfile(fn, dtype=dtype).reshape(chunks)
        sl = tuple(slice(i * c, min((i + 1) * c, s)) for i, c, s in zip(idx, chunks, shape))
        out[sl] = block[tuple(slice(0, x.stop - x.start) for x in sl)]
    return out


def read_attrs(path, name=None):
    with open(os.path.join(path, name, ".zattrs") if name else os.path.join(path, ".zattrs")) as f:
        return json.load(f)
