"""MosaicML-Streaming **MDS** shards: writer + streaming reader (+ native batch assembly).

The reference writes TinyImageNet to MDS with ``MDSWriter(out, columns={'image': 'pil', 'label':
'int'}, compression='zstd')`` (`01_torch_distributor/03a_tiny_imagenet_torch_distributor_resnet_mds.py:179-223`)
and trains from ``TinyImageNetMDS(StreamingDataset)`` (`:240-255`, `:382-393`). mosaicml-streaming
is not installed here, so both sides are implemented from the format:

* ``index.json``: ``{"version": 2, "shards": [{"format": "mds", "version": 2, "samples": n,
  "column_names": [...], "column_encodings": [...], "column_sizes": [...|null],
  "compression": null, "raw_data": {"basename": "shard.00000.mds", "bytes": B, "hashes": {}},
  "size_limit": L, "hashes": [], "zip_data": null}]}``;
* shard file: ``uint32 n``, ``uint32 offsets[n+1]`` (absolute), then samples; a sample is the
  uint32 byte sizes of its variable-size columns followed by every column's bytes in order;
* encodings: ``int`` (int64), ``str``/``bytes``, ``pil`` (uint32 w, h, len(mode) + mode + raw
  pixels), ``jpeg``/``png`` (file bytes), ``ndarray:<dtype>:<d0,d1,...>`` (raw).

Compression (``compression='gz' | 'gz:<level>' | 'bz2' | 'zstd[:<level>]'``): as in mosaicml-streaming,
a compressed shard is stored as ``zip_data`` (``shard.00000.mds.gz`` ...) next to the uncompressed
``raw_data`` description; the reader decompresses it once into its ``local`` directory and then
memory-maps the raw shard (the C++ assembler always reads raw shards). ``gz`` / ``bz2`` use the
standard library; ``zstd`` (the reference's choice, `03a…:195`) goes through the system ``libzstd.so.1``
loaded with ctypes (``ZSTD_compress`` / ``ZSTD_decompress``, GIL released during the call) or the
``zstandard`` module when that is installed; only when neither exists does the writer fall back to
uncompressed shards (with a warning) and the reader raise a clear error for the zstd shards.
Raw ``pil`` pixels are what the native loader wants anyway (no image decode at all). Parity with
mosaicml-streaming's own reader is "unpinned" (not installed); tests pin the format round-trip
(tests/test_data.py).

:class:`StreamingDataset` partitions samples over ``RANK/WORLD_SIZE`` (and DataLoader workers)
deterministically per epoch — no shared-memory coordination.
:meth:`StreamingDataset.native_reader` hands the shard set to the C++ assembler
(``csrc/runtime/mds_loader.cpp``), which gathers a batch of raw ``pil`` images straight into a
pinned uint8 NHWC buffer with a thread pool (``data.loader``).
"""
from __future__ import annotations

import io
import json
import os
import shutil
import struct
from typing import Any, Dict, Iterator, List, Optional, Sequence

import numpy as np
import torch
from torch.utils.data import IterableDataset, get_worker_info

try:
    from PIL import Image
except Exception:  # pragma: no cover
    Image = None

FIXED_SIZES = {"int": 8, "int64": 8, "int32": 4, "float32": 4, "float64": 8, "uint8": 1}


# ---------------------------------------------------------------------------------------
# encodings
# ---------------------------------------------------------------------------------------
def encode(enc: str, obj: Any) -> bytes:
    if enc in ("int", "int64"):
        return np.int64(obj).tobytes()
    if enc == "int32":
        return np.int32(obj).tobytes()
    if enc == "float32":
        return np.float32(obj).tobytes()
    if enc == "float64":
        return np.float64(obj).tobytes()
    if enc == "uint8":
        return np.uint8(obj).tobytes()
    if enc == "str":
        return obj.encode("utf-8")
    if enc == "bytes":
        return bytes(obj)
    if enc == "pil":
        if not isinstance(obj, Image.Image):
            obj = Image.fromarray(np.asarray(obj))
        mode = obj.mode.encode("utf-8")
        w, h = obj.size
        return np.array([w, h, len(mode)], np.uint32).tobytes() + mode + obj.tobytes()
    if enc in ("jpeg", "png"):
        if isinstance(obj, (bytes, bytearray)):
            return bytes(obj)
        if not isinstance(obj, Image.Image):
            obj = Image.fromarray(np.asarray(obj))
        buf = io.BytesIO()
        obj.save(buf, format="JPEG" if enc == "jpeg" else "PNG")
        return buf.getvalue()
    if enc.startswith("ndarray"):
        return np.ascontiguousarray(obj).tobytes()
    raise ValueError(f"unsupported MDS encoding {enc!r}")


def decode(enc: str, data: bytes) -> Any:
    if enc in ("int", "int64"):
        return int(np.frombuffer(data, np.int64)[0])
    if enc == "int32":
        return int(np.frombuffer(data, np.int32)[0])
    if enc == "float32":
        return float(np.frombuffer(data, np.float32)[0])
    if enc == "float64":
        return float(np.frombuffer(data, np.float64)[0])
    if enc == "uint8":
        return int(data[0])
    if enc == "str":
        return data.decode("utf-8")
    if enc == "bytes":
        return data
    if enc == "pil":
        w, h, ml = np.frombuffer(data[:12], np.uint32)
        mode = data[12:12 + ml].decode("utf-8")
        return Image.frombytes(mode, (int(w), int(h)), data[12 + ml:])
    if enc in ("jpeg", "png"):
        return Image.open(io.BytesIO(data))
    if enc.startswith("ndarray"):
        _, dt, shp = enc.split(":")
        return np.frombuffer(data, np.dtype(dt)).reshape([int(x) for x in shp.split(",")])
    raise ValueError(f"unsupported MDS encoding {enc!r}")


def _fixed_size(enc: str) -> Optional[int]:
    if enc in FIXED_SIZES:
        return FIXED_SIZES[enc]
    if enc.startswith("ndarray"):
        _, dt, shp = enc.split(":")
        return int(np.prod([int(x) for x in shp.split(",")])) * np.dtype(dt).itemsize
    return None


# ---------------------------------------------------------------------------------------
# compression codecs (mosaicml-streaming names: "gz", "gz:6", "bz2", "zstd", "zstd:7")
# ---------------------------------------------------------------------------------------
class _LibZstd:
    """The zstd frame format through the system library (ctypes; no headers / package needed)."""
    _UNKNOWN, _ERROR = (1 << 64) - 1, (1 << 64) - 2  # ZSTD_CONTENTSIZE_UNKNOWN / _ERROR

    def __init__(self, lib):
        import ctypes as C
        self.C, self.lib = C, lib
        sz, vp, cp = C.c_size_t, C.c_void_p, C.c_char_p
        lib.ZSTD_compressBound.restype, lib.ZSTD_compressBound.argtypes = sz, [sz]
        lib.ZSTD_compress.restype, lib.ZSTD_compress.argtypes = sz, [vp, sz, vp, sz, C.c_int]
        lib.ZSTD_decompress.restype, lib.ZSTD_decompress.argtypes = sz, [vp, sz, vp, sz]
        lib.ZSTD_getFrameContentSize.restype, lib.ZSTD_getFrameContentSize.argtypes = C.c_ulonglong, [vp, sz]
        lib.ZSTD_isError.restype, lib.ZSTD_isError.argtypes = C.c_uint, [sz]
        lib.ZSTD_getErrorName.restype, lib.ZSTD_getErrorName.argtypes = cp, [sz]

    def _check(self, r: int, what: str) -> int:
        if self.lib.ZSTD_isError(r):
            raise RuntimeError(f"zstd {what}: {self.lib.ZSTD_getErrorName(r).decode()}")
        return r

    def compress(self, data: bytes, level: int = 3) -> bytes:
        cap = self.lib.ZSTD_compressBound(len(data))
        out = self.C.create_string_buffer(cap)
        n = self._check(self.lib.ZSTD_compress(out, cap, data, len(data), int(level)), "compress")
        return out.raw[:n]

    def decompress(self, data: bytes, size: Optional[int] = None) -> bytes:
        fs = self.lib.ZSTD_getFrameContentSize(data, len(data))
        if fs == self._ERROR:
            raise RuntimeError("zstd decompress: not a zstd frame")
        if fs == self._UNKNOWN:
            if size is None:
                raise RuntimeError("zstd decompress: frame without a content size and no size hint")
            fs = size
        out = self.C.create_string_buffer(max(1, fs))
        n = self._check(self.lib.ZSTD_decompress(out, fs, data, len(data)), "decompress")
        return out.raw[:n]


_ZSTD: Any = False


def _libzstd() -> Optional[_LibZstd]:
    global _ZSTD
    if _ZSTD is False:
        _ZSTD = None
        import ctypes
        import ctypes.util
        for name in ("libzstd.so.1", ctypes.util.find_library("zstd") or ""):
            if not name:
                continue
            try:
                _ZSTD = _LibZstd(ctypes.CDLL(name))
                break
            except (OSError, AttributeError):
                continue
    return _ZSTD


def _codec(spec: str, decoder: bool = False):
    """-> (compress fn, file extension), or (extension, decompress fn) with ``decoder=True``."""
    algo, _, lvl = spec.partition(":")
    level = int(lvl) if lvl else None
    if algo == "gz":
        import gzip
        return ("gz", gzip.decompress) if decoder else \
            ((lambda b: gzip.compress(b, compresslevel=9 if level is None else level, mtime=0)), "gz")
    if algo == "bz2":
        import bz2
        return ("bz2", bz2.decompress) if decoder else \
            ((lambda b: bz2.compress(b, 9 if level is None else level)), "bz2")
    if algo == "zstd":
        z = _libzstd()
        if z is not None:
            if decoder:
                return "zstd", z.decompress
            return (lambda b: z.compress(b, 3 if level is None else level)), "zstd"
        try:
            import zstandard
        except ImportError:
            raise RuntimeError(f"MDS compression {spec!r} needs libzstd.so.1 or the zstandard module") from None
        if decoder:
            return "zstd", (lambda b, size=None: zstandard.ZstdDecompressor().decompress(b, max_output_size=size or 0))
        return (lambda b: zstandard.ZstdCompressor(level=3 if level is None else level).compress(b)), "zstd"
    raise RuntimeError(f"unsupported MDS compression {spec!r} (gz, bz2, zstd)")


# ---------------------------------------------------------------------------------------
# writer
# ---------------------------------------------------------------------------------------
class MDSWriter:
    """``with MDSWriter(out=dir, columns={'image': 'pil', 'label': 'int'}) as w: w.write(sample)``."""

    def __init__(self, out: str, columns: Dict[str, str], compression: Optional[str] = None,
                 size_limit: int = 1 << 26, exist_ok: bool = True, **_):
        self.compression = None
        if compression not in (None, "", "none"):
            try:
                _codec(compression)
                self.compression = compression
            except RuntimeError as e:  # zstd without the zstandard module: raw shards, say so once
                import warnings
                warnings.warn(f"{e}; writing uncompressed shards")
        self.out = out
        os.makedirs(out, exist_ok=exist_ok)
        self.names = sorted(columns)
        self.encs = [columns[n] for n in self.names]
        self.sizes = [_fixed_size(e) for e in self.encs]
        self.size_limit = size_limit
        self.shards: List[Dict] = []
        self._samples: List[bytes] = []
        self._bytes = 0

    def write(self, sample: Dict[str, Any]) -> None:
        parts, heads = [], []
        for n, e, sz in zip(self.names, self.encs, self.sizes):
            b = encode(e, sample[n])
            if sz is None:
                heads.append(struct.pack("<I", len(b)))
            elif len(b) != sz:
                raise ValueError(f"column {n}: encoded {len(b)} bytes, expected {sz}")
            parts.append(b)
        rec = b"".join(heads) + b"".join(parts)
        if self._samples and self._bytes + len(rec) + 4 * (len(self._samples) + 2) > self.size_limit:
            self._flush()
        self._samples.append(rec)
        self._bytes += len(rec)

    def _flush(self) -> None:
        if not self._samples:
            return
        n = len(self._samples)
        base = 4 + 4 * (n + 1)
        offs = [base]
        for r in self._samples:
            offs.append(offs[-1] + len(r))
        name = f"shard.{len(self.shards):05d}.mds"
        raw = b"".join([struct.pack("<I", n), np.array(offs, np.uint32).tobytes()] + self._samples)
        zip_data = None
        if self.compression:
            comp, ext = _codec(self.compression)
            zname = f"{name}.{ext}"
            blob = comp(raw)
            with open(os.path.join(self.out, zname), "wb") as f:
                f.write(blob)
            zip_data = {"basename": zname, "bytes": len(blob), "hashes": {}}
        else:
            with open(os.path.join(self.out, name), "wb") as f:
                f.write(raw)
        self.shards.append({
            "column_encodings": self.encs, "column_names": self.names, "column_sizes": self.sizes,
            "compression": self.compression, "format": "mds", "hashes": [],
            "raw_data": {"basename": name, "bytes": offs[-1], "hashes": {}},
            "samples": n, "size_limit": self.size_limit, "version": 2, "zip_data": zip_data,
        })
        self._samples, self._bytes = [], 0

    def finish(self) -> None:
        self._flush()
        with open(os.path.join(self.out, "index.json"), "w") as f:
            json.dump({"shards": self.shards, "version": 2}, f, sort_keys=True)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.finish()
        return False


# ---------------------------------------------------------------------------------------
# reader
# ---------------------------------------------------------------------------------------
class _Shard:
    def __init__(self, path: str, info: Dict):
        self.path = path
        self.info = info
        self.n = info["samples"]
        self.names = info["column_names"]
        self.encs = info["column_encodings"]
        self.sizes = info["column_sizes"]
        self._mm = None
        self._offs = None

    def _open(self):
        if self._mm is None:
            self._mm = np.memmap(self.path, dtype=np.uint8, mode="r")
            n = int(self._mm[:4].view(np.uint32)[0])
            if n != self.n:
                raise ValueError(f"{self.path}: header says {n} samples, index says {self.n}")
            self._offs = self._mm[4:4 + 4 * (n + 1)].view(np.uint32)

    def get_bytes(self, i: int) -> bytes:
        self._open()
        return bytes(self._mm[int(self._offs[i]):int(self._offs[i + 1])])

    def get(self, i: int) -> Dict[str, Any]:
        raw = self.get_bytes(i)
        nvar = sum(1 for s in self.sizes if s is None)
        var_sizes = list(struct.unpack(f"<{nvar}I", raw[:4 * nvar])) if nvar else []
        pos, vi, out = 4 * nvar, 0, {}
        for n, e, s in zip(self.names, self.encs, self.sizes):
            if s is None:
                s = var_sizes[vi]
                vi += 1
            out[n] = decode(e, raw[pos:pos + s])
            pos += s
        return out


class StreamingDataset(IterableDataset):
    """Subset of mosaicml-streaming's StreamingDataset: ``remote`` (copied to ``local``), shuffle,
    deterministic rank / worker partitioning, ``set_epoch``, global ``__getitem__``."""

    def __init__(self, remote: Optional[str] = None, local: Optional[str] = None, shuffle: bool = False,
                 batch_size: Optional[int] = None, shuffle_seed: int = 9176, drop_last: bool = False, **_):
        if local is None and remote is None:
            raise ValueError("need remote and/or local")
        self.local = local or remote
        if remote and local and os.path.abspath(remote) != os.path.abspath(local):
            os.makedirs(local, exist_ok=True)
            for fn in os.listdir(remote):
                src, dst = os.path.join(remote, fn), os.path.join(local, fn)
                if os.path.isfile(src) and (not os.path.exists(dst) or os.path.getsize(dst) != os.path.getsize(src)):
                    shutil.copy2(src, dst)
        with open(os.path.join(self.local, "index.json")) as f:
            idx = json.load(f)
        self.shards: List[_Shard] = []
        for sh in idx["shards"]:
            raw_path = os.path.join(self.local, sh["raw_data"]["basename"])
            if sh.get("compression") and not (os.path.exists(raw_path)
                                              and os.path.getsize(raw_path) == sh["raw_data"]["bytes"]):
                ext, dec = _codec(sh["compression"], decoder=True)
                with open(os.path.join(self.local, sh["zip_data"]["basename"]), "rb") as f:
                    data = dec(f.read(), sh["raw_data"]["bytes"]) if ext == "zstd" else dec(f.read())
                if len(data) != sh["raw_data"]["bytes"]:
                    raise ValueError(f"{sh['zip_data']['basename']}: decompressed {len(data)} bytes, "
                                     f"index says {sh['raw_data']['bytes']}")
                tmp = raw_path + f".tmp{os.getpid()}"
                with open(tmp, "wb") as f:
                    f.write(data)
                os.replace(tmp, raw_path)  # atomic: concurrent local ranks may race to decompress
            self.shards.append(_Shard(raw_path, sh))
        self.cum = np.cumsum([0] + [s.n for s in self.shards])
        self.num_samples = int(self.cum[-1])
        self.shuffle, self.seed, self.batch_size, self.drop_last = shuffle, shuffle_seed, batch_size, drop_last
        self.epoch = 0
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def locate(self, idx: int):
        s = int(np.searchsorted(self.cum, idx, side="right") - 1)
        return s, idx - int(self.cum[s])

    def get_item(self, idx: int) -> Dict[str, Any]:
        s, i = self.locate(idx)
        return self.shards[s].get(i)

    def __getitem__(self, idx: int):
        return self.get_item(idx)

    def epoch_indices(self) -> np.ndarray:
        """This rank's sample ids for the current epoch (padded by wrap-around to equal length)."""
        n = self.num_samples
        order = np.random.default_rng(self.seed + self.epoch).permutation(n) if self.shuffle else np.arange(n)
        per = n // self.world if self.drop_last else -(-n // self.world)
        total = per * self.world
        if total > n:
            order = np.concatenate([order, order[:total - n]])
        return order[self.rank:total:self.world]

    def __len__(self) -> int:
        n = self.num_samples
        return n // self.world if self.drop_last else -(-n // self.world)

    def __iter__(self) -> Iterator:
        ids = self.epoch_indices()
        wi = get_worker_info()
        if wi is not None:
            ids = ids[wi.id::wi.num_workers]
        for i in ids:
            yield self[int(i)]

    def native_reader(self):
        """C++ batch assembler over these shards (``_C.MDSReader``)."""
        from ..ops._ext import C
        return C().MDSReader([s.path for s in self.shards], [s.n for s in self.shards],
                             self.shards[0].names, self.shards[0].encs,
                             [(-1 if z is None else int(z)) for z in self.shards[0].sizes])


def write_image_dataset_mds(dataset, out: str, image_key: str = "image", label_key: str = "label",
                            encoding: str = "pil", size_limit: int = 1 << 26, limit: Optional[int] = None) -> int:
    """Serialise an (image, label) dataset (PIL / uint8 HWC images) to MDS (03a's writer loop)."""
    n = 0
    with MDSWriter(out, {image_key: encoding, label_key: "int"}, size_limit=size_limit) as w:
        for i in range(len(dataset)):
            if limit is not None and i >= limit:
                break
            img, y = dataset[i]
            if isinstance(img, np.ndarray):
                img = Image.fromarray(img if img.ndim == 2 or img.shape[2] != 1 else img[..., 0])
            w.write({image_key: img, label_key: int(y)})
            n += 1
    return n
