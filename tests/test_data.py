"""Data subsystem: MDS round trip (python + native C++ reader), sampler, transforms, IDX/CIFAR readers."""
import os
import tempfile

import numpy as np
import pytest
import torch

from dbx_distributed_pytorch_examples_amd.data import transforms as T
from dbx_distributed_pytorch_examples_amd.data.datasets import (CIFAR10, MNIST, SyntheticImages, write_cifar10_bin,
                                                                write_idx)
from dbx_distributed_pytorch_examples_amd.data.loader import AugmentSpec, NativeImageLoader, sample_boxes
from dbx_distributed_pytorch_examples_amd.data.mds import MDSWriter, StreamingDataset, write_image_dataset_mds
from dbx_distributed_pytorch_examples_amd.parallel.sampler import ShardSampler


def _mds(tmp, n=37, size=8, limit=2000):
    ds = SyntheticImages(n, size, 3, 10, seed=3)
    write_image_dataset_mds(ds, tmp, size_limit=limit)
    return ds


def test_mds_roundtrip_and_shards():
    d = tempfile.mkdtemp()
    ds = _mds(d)
    sd = StreamingDataset(local=d)
    assert sd.num_samples == 37 and len(sd.shards) > 1
    for i in (0, 5, 36):
        it = sd[i]
        assert np.array_equal(np.asarray(it["image"]), ds[i][0])
        assert it["label"] == ds[i][1]


@pytest.mark.parametrize("comp", ["gz", "gz:1", "bz2", "zstd", "zstd:7"])
def test_mds_compressed_shards(comp):
    """compressed shards (zip_data next to raw_data, as mosaicml-streaming writes them) are
    decompressed once into the reader's local directory; remote keeps only the compressed files"""
    import json
    remote, local = tempfile.mkdtemp(), tempfile.mkdtemp()
    ds = SyntheticImages(23, 8, 3, 10, seed=4)
    with MDSWriter(remote, {"image": "pil", "label": "int"}, compression=comp, size_limit=1500) as w:
        for i in range(len(ds)):
            img, y = ds[i]
            w.write({"image": img, "label": y})
    idx = json.load(open(os.path.join(remote, "index.json")))
    ext = comp.split(":")[0]
    assert len(idx["shards"]) > 1
    for sh in idx["shards"]:
        assert sh["compression"] == comp and sh["zip_data"]["basename"].endswith("." + ext)
        assert not os.path.exists(os.path.join(remote, sh["raw_data"]["basename"]))
    sd = StreamingDataset(remote=remote, local=local)
    assert sd.num_samples == 23
    for i in (0, 11, 22):
        assert np.array_equal(np.asarray(sd[i]["image"]), ds[i][0]) and sd[i]["label"] == ds[i][1]
    sd2 = StreamingDataset(local=local)  # second open: raw shards already materialised
    assert np.array_equal(np.asarray(sd2[5]["image"]), ds[5][0])


def test_mds_zstd_frames_roundtrip():
    """zstd through the system libzstd (ctypes): standard frames with the content size, and a
    frame without one decoded with the index's raw size as the hint."""
    from dbx_distributed_pytorch_examples_amd.data import mds
    z = mds._libzstd()
    if z is None:
        pytest.skip("no libzstd.so.1 on this host")
    data = bytes(range(256)) * 999 + b"tail"
    c = z.compress(data, 5)
    assert c[:4] == b"\x28\xb5\x2f\xfd" and len(c) < len(data) // 10  # zstd magic, compressed
    assert z.decompress(c) == data
    with pytest.raises(RuntimeError, match="not a zstd frame"):
        z.decompress(b"garbage!")


def test_mds_zstd_without_any_codec_falls_back(monkeypatch):
    from dbx_distributed_pytorch_examples_amd.data import mds
    monkeypatch.setattr(mds, "_ZSTD", None)  # as if libzstd were missing
    try:
        import zstandard  # noqa: F401
        pytest.skip("zstandard installed: the fallback path is not taken")
    except ImportError:
        pass
    d = tempfile.mkdtemp()
    with pytest.warns(UserWarning, match="zstandard"):
        w = MDSWriter(d, {"label": "int"}, compression="zstd")
    w.write({"label": 3})
    w.finish()
    assert StreamingDataset(local=d)[0]["label"] == 3


def test_mds_mixed_columns():
    d = tempfile.mkdtemp()
    with MDSWriter(d, {"a": "int", "s": "str", "b": "bytes", "x": "ndarray:float32:2,3"}) as w:
        for i in range(5):
            w.write({"a": i, "s": "x" * i, "b": bytes([i] * i), "x": np.full((2, 3), i, np.float32)})
    sd = StreamingDataset(local=d)
    it = sd[4]
    assert it["a"] == 4 and it["s"] == "xxxx" and it["b"] == bytes([4] * 4) and it["x"].sum() == 24


def test_mds_rank_partition(monkeypatch):
    d = tempfile.mkdtemp()
    _mds(d, n=10)
    seen = []
    for r in range(3):
        monkeypatch.setenv("RANK", str(r))
        monkeypatch.setenv("WORLD_SIZE", "3")
        sd = StreamingDataset(local=d, shuffle=True)
        ids = sd.epoch_indices()
        assert len(ids) == 4
        seen.extend(ids.tolist())
    assert set(seen) == set(range(10))


def test_mds_native_reader():
    from dbx_distributed_pytorch_examples_amd.ops import _ext
    if not _ext.available():
        pytest.skip("extension not built")
    d = tempfile.mkdtemp()
    ds = _mds(d, n=20, size=16)
    sd = StreamingDataset(local=d)
    rd = sd.native_reader()
    assert rd.num_samples() == 20
    idx = np.array([3, 0, 19, 7], np.int64)
    out = torch.empty(4, 16, 16, 3, dtype=torch.uint8)
    lab = torch.empty(4, dtype=torch.int64)
    rd.gather(idx, out.data_ptr(), lab.data_ptr(), 16, 16, 3, "image", "label", 3)
    for k, i in enumerate(idx):
        assert np.array_equal(out[k].numpy(), ds[int(i)][0])
        assert lab[k].item() == ds[int(i)][1]
    with pytest.raises(RuntimeError):
        rd.gather(idx, out.data_ptr(), lab.data_ptr(), 8, 8, 3, "image", "label", 2)


def test_native_loader_cpu():
    d = tempfile.mkdtemp()
    _mds(d, n=24, size=16)
    sd = StreamingDataset(local=d)
    ld = NativeImageLoader(sd, 8, (16, 16), torch.device("cpu"), augment=AugmentSpec(mode="random_crop", pad=2, hflip=True),
                           out_hw=(12, 12), nthreads=2)
    batches = list(ld)
    assert len(batches) == 3
    img, lab, boxes, flips = batches[0]
    assert img.shape == (8, 16, 16, 3) and img.dtype == torch.uint8 and boxes.shape == (8, 4)


def test_sampler_matches_torch_semantics():
    s = [ShardSampler(10, num_replicas=3, rank=r, shuffle=True, seed=1) for r in range(3)]
    allidx = sum((list(x) for x in s), [])
    assert len(allidx) == 12 and set(allidx) == set(range(10))
    s[0].set_epoch(1)
    assert list(s[0]) != list(ShardSampler(10, 3, 0, True, 1))
    d = ShardSampler(10, 3, 0, drop_last=True)
    assert len(d) == 3


def test_sample_boxes_modes():
    import random
    rng = random.Random(0)
    b, f = sample_boxes(16, 256, 256, 224, 224, AugmentSpec(mode="random_resized_crop", hflip=True), rng)
    assert (b[:, 2] <= 256).all() and (b[:, 3] <= 256).all() and set(f.tolist()) <= {0, 1}
    b, _ = sample_boxes(4, 256, 256, 224, 224, AugmentSpec(mode="center_crop"), rng)
    assert np.allclose(b[0], [16, 16, 224, 224])


def test_transforms_pipeline():
    img = (np.random.rand(40, 30, 3) * 255).astype(np.uint8)
    t = T.default_image_transforms(32)
    x = t(img)
    assert x.shape == (3, 32, 32)
    assert T.cifar_transforms(True)(np.zeros((32, 32, 3), np.uint8)).shape == (3, 32, 32)
    assert T.imagenet_transforms(True)(img).shape == (3, 224, 224)
    g = T.default_image_transforms(16, grayscale_first=True)(np.zeros((20, 20), np.uint8))
    assert g.shape == (3, 16, 16)


def test_idx_and_cifar_readers():
    d = tempfile.mkdtemp()
    imgs = (np.random.rand(5, 28, 28) * 255).astype(np.uint8)
    write_idx(os.path.join(d, "train-images-idx3-ubyte"), imgs)
    write_idx(os.path.join(d, "train-labels-idx1-ubyte"), np.arange(5, dtype=np.uint8))
    m = MNIST(d, train=True)
    assert len(m) == 5 and m[3][1] == 3 and np.array_equal(m[2][0][..., 0], imgs[2])
    c_imgs = (np.random.rand(6, 32, 32, 3) * 255).astype(np.uint8)
    for i in range(1, 6):
        write_cifar10_bin(os.path.join(d, f"data_batch_{i}.bin"), c_imgs, np.arange(6) % 10)
    c = CIFAR10(d, train=True)
    assert len(c) == 30 and np.array_equal(c[1][0], c_imgs[1]) and c[1][1] == 1


def test_learnable_synthetic_is_deterministic_and_class_structured():
    import torch
    from dbx_distributed_pytorch_examples_amd.data.datasets import learnable_synthetic
    x1, y1 = learnable_synthetic(256, 32, 10, seed=3)
    x2, y2 = learnable_synthetic(256, 32, 10, seed=3)
    assert x1.shape == (256, 32, 32, 3) and x1.dtype == torch.uint8
    assert torch.equal(x1, x2) and torch.equal(y1, y2)
    # nearest-class-mean on the held-out split beats chance by a wide margin (the task is learnable)
    xv, yv = learnable_synthetic(256, 32, 10, seed=4)
    means = torch.stack([x1[y1 == c].float().mean(0) for c in range(10)])
    d = ((xv.float()[:, None] - means[None]) ** 2).flatten(2).sum(-1)
    acc = (d.argmin(1) == yv).float().mean().item()
    assert acc > 0.3, acc


def test_hf_dataset_class_pickles_with_the_standard_pickler():
    """create_torch_image_dataset's class and instances survive plain pickle, also in a fresh process
    that never created the class (spawn DataLoader workers, launcher children)."""
    import pickle
    import subprocess
    import sys
    from dbx_distributed_pytorch_examples_amd.data.hf import create_torch_image_dataset
    cls = create_torch_image_dataset("img", "fine label")
    assert create_torch_image_dataset("img", "fine label") is cls
    ds = cls({"img": [1, 2, 3], "fine label": [0, 1, 1]})
    blob = pickle.dumps(ds)
    back = pickle.loads(blob)
    assert type(back) is cls and back[2] == (3, 1) and back.num_classes == 2
    assert pickle.loads(pickle.dumps(cls)) is cls
    code = ("import pickle, sys; ds = pickle.loads(sys.stdin.buffer.read()); "
            "print(type(ds).image_key, type(ds).label_key, len(ds), ds[1])")
    r = subprocess.run([sys.executable, "-c", code], input=blob, capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    assert r.stdout.decode().strip() == "img fine label 3 (2, 1)"
