"""Streaming writer for ray histories.

The reference's lightsheet sweep (scripts/2024_04_01_lightsheet.py:53-60, 134-135) stores one history
per configuration in a zarr array ``rays`` of shape (n_config, planes, n_rays, 8) chunked one
configuration per chunk, with ``array_columns`` = x, y, z, dx, dy, dz, phase, wavelength.  zarr is
not a dependency here, so :class:`HistoryWriter` writes that exact layout as a zarr-v2 directory store
itself (``.zarray`` / ``.zattrs`` / ``.zgroup`` JSON), readable by zarr when it is installed and by
:func:`read_array` otherwise.  Chunks are stored raw (``compressor: null``) or compressed with zlib (zarr's
``numcodecs.Zlib``: ``{"id": "zlib", "level": L}``, each chunk one ``zlib.compress`` stream); a configuration may be
split along the ray axis (``chunk_rays``) so its chunks compress on several threads.  The script's own store uses
zarr's default Blosc/LZ4 compressor, which needs the c-blosc library (not installed here): the compressed variant
is a different, zarr-readable codec, and its parity is pinned only by this module's round trips.

Histories may be NumPy arrays or torch CUDA tensors.  Device histories are copied into pinned host
buffers on a side stream and written by a background thread, so the GPU can trace the next
configuration while the previous one goes to disk (double-buffered).
"""
import concurrent.futures
import json
import os
import queue
import threading
import zlib

import numpy as np

from . import _engine as E

ARRAY_COLUMNS = ["x", "y", "z", "dx", "dy", "dz", "phase", "wavelength"]


def _zarray(shape, chunks, dtype, compressor=None):
    return {"zarr_format": 2, "shape": list(shape), "chunks": list(chunks), "dtype": np.dtype(dtype).str,
            "compressor": compressor, "fill_value": "NaN" if np.dtype(dtype).kind == "f" else 0, "filters": None,
            "order": "C", "dimension_separator": "."}


def _codec(compressor):
    """The zarr compressor metadata for `compressor`: None (raw chunks), "zlib" (level 1), ("zlib", level) or a
    numcodecs-style dict {"id": "zlib", "level": level}."""
    if compressor is None:
        return None
    if isinstance(compressor, str):
        compressor = (compressor, 1)
    if isinstance(compressor, (tuple, list)):
        compressor = {"id": compressor[0], "level": int(compressor[1])}
    compressor = dict(compressor)
    if compressor.get("id") != "zlib" or not 0 <= int(compressor.get("level", 1)) <= 9:
        raise ValueError(f"unsupported compressor {compressor!r} (None or zlib level 0-9)")
    return {"id": "zlib", "level": int(compressor.get("level", 1))}


def _encode(codec, raw):
    return raw if codec is None else zlib.compress(raw, codec["level"])


def _decode(codec, data):
    if codec is None:
        return data
    if codec.get("id") != "zlib":
        raise ValueError(f"unsupported compressor {codec!r}")
    return zlib.decompress(data)


def _write_json(path, obj):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f, indent=1)
    os.replace(tmp, path)


class HistoryWriter:
    """zarr-v2 store at ``path`` with array ``rays`` (n_configs, n_planes, n_rays, 8).

    compressor: None (raw chunks, the default), "zlib", ("zlib", level) or {"id": "zlib", "level": level}.
    chunk_rays: rays per chunk (default: all -- one chunk per configuration, the script's chunks=(1, planes,
    nrays, 8)); the last chunk of a configuration is stored at full chunk size, padded with the fill value (NaN),
    as zarr stores edge chunks.  workers: threads encoding and writing chunks; compressed configurations with fewer
    chunks than workers are encoded up to ``depth`` at a time (raw ones one at a time)."""

    def __init__(self, path, n_configs, n_planes, n_rays, dtype="float64", attrs=None, depth=2, compressor=None,
                 chunk_rays=None, workers=None):
        self.path = str(path)
        self.shape = (int(n_configs), int(n_planes), int(n_rays), 8)
        self.dtype = np.dtype(dtype)
        self.codec = _codec(compressor)
        self.chunk_rays = int(chunk_rays) if chunk_rays else max(self.shape[2], 1)
        if self.chunk_rays < 1:
            raise ValueError("chunk_rays must be positive")
        os.makedirs(os.path.join(self.path, "rays"), exist_ok=True)
        _write_json(os.path.join(self.path, ".zgroup"), {"zarr_format": 2})
        _write_json(os.path.join(self.path, ".zattrs"), dict(attrs or {}))
        _write_json(os.path.join(self.path, "rays", ".zarray"),
                    _zarray(self.shape, (1, self.shape[1], self.chunk_rays, 8), self.dtype, self.codec))
        _write_json(os.path.join(self.path, "rays", ".zattrs"), {"array_columns": ARRAY_COLUMNS})
        self._n_chunks = -(-self.shape[2] // self.chunk_rays)
        n_workers = max(1, int(workers or min(8, os.cpu_count() or 1)))
        self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=n_workers)
        # configurations whose chunks are encoded at once (each holds its host copy until written): raw chunks one
        # at a time, as the disk takes them; compressed ones up to `depth`, enough to keep the workers busy when a
        # configuration has fewer chunks than there are workers
        inflight = 1 if self.codec is None else max(1, min(int(depth), -(-n_workers // max(self._n_chunks, 1))))
        self._inflight = threading.BoundedSemaphore(inflight)
        self._q = queue.Queue(maxsize=depth)
        self._free = queue.Queue()
        self._err = None
        self._pinned = []
        self._thread = threading.Thread(target=self._drain, daemon=True)
        self._thread.start()

    # -------------------------------------------------------------------- chunks
    def _chunk_file(self, index, j=0):
        return os.path.join(self.path, "rays", f"{index}.0.{j}.0")

    def _write_chunk(self, index, j, arr):
        """Chunk j of configuration `index` (rays j*chunk_rays ...), padded to the chunk shape, encoded, written
        atomically (zlib releases the GIL: the pool's threads compress in parallel)."""
        c = self.chunk_rays
        block = arr[:, j * c:(j + 1) * c]
        if block.shape[1] < c:
            pad = np.full((block.shape[0], c, 8), np.nan if self.dtype.kind == "f" else 0, dtype=self.dtype)
            pad[:, :block.shape[1]] = block
            block = pad
        data = _encode(self.codec, memoryview(np.ascontiguousarray(block)).cast("B"))
        tmp = self._chunk_file(index, j) + ".tmp"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, self._chunk_file(index, j))

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
            except Exception as e:  # surfaced by the next write()/close()
                self._err = e
                if buf is not None:
                    self._free.put(buf)
                continue
            if self._n_chunks == 0:
                if buf is not None:
                    self._free.put(buf)
                continue
            # the configuration's chunks go to the pool; its host copy returns to the free list when the last one
            # is written, and the semaphore bounds the configurations in flight (and so the host copies held)
            self._inflight.acquire()
            left = [self._n_chunks]
            lock = threading.Lock()

            def done(fut, buf=buf):
                if fut.exception() is not None:
                    self._err = fut.exception()
                with lock:
                    left[0] -= 1
                    last = left[0] == 0
                if last:
                    if buf is not None:
                        self._free.put(buf)
                    self._inflight.release()
            for j in range(self._n_chunks):
                self._pool.submit(self._write_chunk, index, j, arr).add_done_callback(done)

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
        self._pool.shutdown(wait=True)
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
    codec = meta.get("compressor")
    out = np.full(shape, fill, dtype=dtype)
    grid = [range(-(-s // c)) for s, c in zip(shape, chunks)]
    for idx in np.ndindex(*[len(g) for g in grid]):
        fn = os.path.join(path, name, ".".join(str(i) for i in idx) if idx else "0")
        if not os.path.exists(fn):
            continue
        with open(fn, "rb") as f:
            block = np.frombuffer(_decode(codec, f.read()), dtype=dtype).reshape(chunks)
        sl = tuple(slice(i * c, min((i + 1) * c, s)) for i, c, s in zip(idx, chunks, shape))
        out[sl] = block[tuple(slice(0, x.stop - x.start) for x in sl)]
    return out


def read_attrs(path, name=None):
    with open(os.path.join(path, name, ".zattrs") if name else os.path.join(path, ".zattrs")) as f:
        return json.load(f)
