"""CPU tests: config system, schedules, MLflow-compatible tracking, checkpoints, profiling and
debug utilities, bootstrap, inference helpers, dataset snapshots."""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

from dbx_distributed_pytorch_examples_amd import bootstrap, config
from dbx_distributed_pytorch_examples_amd.data.datasets import SyntheticImages, TensorImageDataset, save_tensor_dataset
from dbx_distributed_pytorch_examples_amd.frontends import deepspeed as dsf
from dbx_distributed_pytorch_examples_amd.train.schedule import LRSchedule, linear_scaled_lr
from dbx_distributed_pytorch_examples_amd.utils import checkpoint as ckpt
from dbx_distributed_pytorch_examples_amd.utils import debug, inference, profiling


# ---------------------------------------------------------------------------------- config
def test_config_yaml_overrides_and_durations(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("model: resnet18\nbatch_size: 32\noptim:\n  name: adamw\n  lr: 0.002\n")
    cfg = config.load_config(str(p), overrides=["epochs=3", "optim.weight_decay=0.05", "graphs=false"])
    assert cfg.model == "resnet18" and cfg.batch_size == 32 and cfg.epochs == 3
    assert cfg.optim.name == "adamw" and cfg.optim.lr == 0.002 and cfg.optim.weight_decay == 0.05
    assert cfg.graphs is False
    assert config.parse_duration("2ep", 100) == 200
    assert config.parse_duration("150ba", 100) == 150
    assert config.parse_duration("5000sp", 100, batch_size=50) == 100
    with pytest.raises(Exception):
        config.apply_overrides(cfg, ["no_such_key=1"])


def test_local_config_volumes(tmp_path):
    p = tmp_path / "local_config.yaml"
    p.write_text("catalog: cat\nschema: sch\ncifar_cache: /Volumes/cat/sch/cifar\nnum_nodes: 2\n")
    lc = config.load_local_config(str(p))
    lc.volume_root = str(tmp_path / "vol")
    assert lc.num_nodes == 2
    assert lc.volume("cifar_cache").endswith(os.path.join("cat", "sch", "cifar"))
    assert lc.volume("imagenet1k_cache") == os.path.join(str(tmp_path / "vol"), "cat", "sch", "imagenet_1k")


def test_deepspeed_configs_map_to_engine():
    cfg = config.from_deepspeed(dsf.zero_1)
    assert cfg.precision == "bf16" and cfg.optim.name == "adamw" and cfg.optim.lr == 2e-4
    assert cfg.optim.grad_clip == 0.3 and cfg.batch_size == 4
    assert cfg.sched.name == "warmup_lr" and cfg.sched.warmup_steps == 100
    assert cfg.zero.stage == 1 and cfg.zero.reduce_scatter
    assert config.from_deepspeed(dsf.zero_2).zero.stage == 2
    z3 = config.from_deepspeed(dsf.zero_3_offload)
    assert z3.zero.stage == 3 and z3.zero.offload_optimizer


# ---------------------------------------------------------------------------------- schedule
def test_schedules():
    assert linear_scaled_lr(0.1, 8192) == pytest.approx(3.2)
    s = LRSchedule("warmup_cosine", 1.0, total_steps=110, warmup_steps=10)
    assert s(0) == pytest.approx(0.1) and s(9) == pytest.approx(1.0)
    assert s(10) == pytest.approx(1.0) and s(109) < 0.01
    c = LRSchedule("cosine", 1.0, steps_per_epoch=10, t_max_epochs=4)
    assert c(0) == 1.0 and c(20) == pytest.approx(0.5) and c(40) == pytest.approx(0.0, abs=1e-12)
    w = LRSchedule("warmup_lr", 2e-4, warmup_steps=100, warmup_min_lr=0.0)
    assert w(0) == 0.0 and w(99) == pytest.approx(2e-4) and w(500) == 2e-4
    st = LRSchedule("step", 1.0, steps_per_epoch=1, step_size=30, gamma=0.1)
    assert st(29) == 1.0 and st(30) == pytest.approx(0.1)


# ---------------------------------------------------------------------------------- mlflow
def test_mlflow_compat_roundtrip(tmp_path, monkeypatch):
    from dbx_distributed_pytorch_examples_amd.utils import mlflow_compat as mlflow
    monkeypatch.setenv("MLFLOW_TRACKING_URI", "file:" + str(tmp_path / "mlruns"))
    mlflow.set_experiment("/Users/me/experiments/nb")
    with mlflow.start_run(run_name="r") as run:
        mlflow.log_params({"lr": 0.1, "bs": 8})
        for i in range(3):
            mlflow.log_metric("train_loss", 1.0 / (i + 1), step=i)
        mlflow.log_metrics({"val/acc": 0.5})
        mlflow.log_dict({"a": 1}, "meta/info.json")
        m = nn.Linear(3, 2)
        mlflow.pytorch.log_model(m, "model")
        mlflow.pytorch.log_state_dict({"w": torch.ones(2)}, "checkpoints/epoch_1")
        rid = run.info.run_id
    hist = mlflow.get_metric_history(rid, "train_loss")
    assert [(step, v) for step, v, _ts in hist] == [(0, 1.0), (1, 0.5), (2, pytest.approx(1 / 3))]
    assert mlflow.get_params(rid)["lr"] == "0.1"
    m2 = mlflow.pytorch.load_model(f"runs:/{rid}/model")
    assert torch.allclose(m2.weight, m.weight)
    sd = mlflow.pytorch.load_state_dict(f"runs:/{rid}/checkpoints/epoch_1")
    assert torch.equal(sd["w"], torch.ones(2))


# ---------------------------------------------------------------------------------- checkpoints
def test_checkpoint_layouts(tmp_path):
    m = nn.Sequential(nn.Linear(4, 3))
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    m(torch.randn(2, 4)).sum().backward()
    opt.step()
    for e in (1, 2):
        ckpt.save_checkpoint(str(tmp_path), m, opt, epoch=e)
    assert ckpt.latest_checkpoint(str(tmp_path)).endswith("checkpoint-2.pth.tar")
    st = ckpt.load_checkpoint(str(tmp_path), epoch=2)
    assert set(st["model"]) == {"0.weight", "0.bias"} and "optimizer" in st
    a = ckpt.accelerate_checkpoint(3, m, opt, None, test_accuracy=0.7)
    assert a["epoch"] == 3 and "model_state_dict" in a and a["test_accuracy"] == 0.7
    d = tmp_path / "ray"
    ckpt.save_ray_checkpoint(str(d), m)
    assert set(ckpt.load_ray_checkpoint(str(d))) == {"0.weight", "0.bias"}


# ---------------------------------------------------------------------------------- profiling
def test_phase_timer_and_rocprof_helpers(tmp_path):
    t = profiling.PhaseTimer(use_cuda=False)
    for _ in range(3):
        with t.phase("fwd"):
            sum(range(1000))
        with t.phase("bwd"):
            pass
    s = t.summary()
    assert s["fwd"]["count"] == 3 and s["bwd"]["mean_ms"] >= 0
    with profiling.range("outer"):
        profiling.mark("m")
    cmd = profiling.rocprof_cmd(["python3", "bench.py"], "out", pmc=profiling.PMC_GROUPS["mfma"])
    assert cmd[0] == "rocprofv3" and "--pmc" in cmd and cmd[cmd.index("--") + 1] == "python3"
    assert "--sys-trace" not in cmd and "--kernel-trace" not in cmd  # counters stay in their own pass
    csvp = tmp_path / "run_kernel_stats.csv"
    csvp.write_text('"Name","Calls","TotalDurationNs","AverageNs","Percentage"\n'
                    '"k1",10,3000000,300000,75\n"k2",5,1000000,200000,25\n')
    rows = profiling.summarize_kernel_stats(str(tmp_path), steps=2)
    assert rows[0]["name"] == "k1" and rows[0]["ms_per_step"] == pytest.approx(1.5)
    cc = tmp_path / "c" / "run_counter_collection.csv"
    cc.parent.mkdir()
    cc.write_text('"Kernel_Name","Counter_Name","Counter_Value"\n"g","SQ_BUSY_CYCLES",100\n'
                  '"g","SQ_VALU_MFMA_BUSY_CYCLES",250\n"g","SQ_INSTS_MFMA",10\n"g","SQ_INSTS_VALU",30\n')
    d = profiling.summarize_counters(str(tmp_path / "c"))
    assert d["g"]["valu_per_mfma"] == pytest.approx(3.0) and d["g"]["mfma_busy_per_busy"] == 2.5


def test_committed_profiles_parse():
    root = os.path.join(os.path.dirname(__file__), "..", "profiles")
    found = [os.path.join(dp, f) for dp, _, fs in os.walk(root) for f in fs if f.endswith("kernel_stats.csv")]
    assert found, "profiles/ must hold rocprofv3 kernel stats"
    rows = profiling.summarize_kernel_stats(found[0])
    assert rows and rows[0]["ms_per_step"] > 0


# ---------------------------------------------------------------------------------- debug
def test_debug_helpers(monkeypatch):
    env = debug.debug_env(2)
    assert env["AMD_SERIALIZE_KERNEL"] == "3" and env["NCCL_DEBUG"] == "INFO"
    a = [torch.ones(3), torch.arange(4.0)]
    b = [torch.ones(3), torch.arange(4.0).flip(0)]
    assert not torch.equal(debug.replica_checksum(a), debug.replica_checksum(b))  # order sensitive
    debug.assert_replicas_in_sync(a)  # world 1: no-op
    debug.check_bucket_order([2, 1, 0])

    @debug.checked_op
    def op(x):
        return x * 2

    monkeypatch.setenv("DBX_DEBUG", "1")
    assert debug.enabled()
    assert torch.equal(op(torch.ones(2)), torch.full((2,), 2.0))  # CPU tensors: no device sync


# ---------------------------------------------------------------------------------- bootstrap
def test_bootstrap_setup(tmp_path, monkeypatch):
    lc = tmp_path / "local_config.yaml"
    lc.write_text(f"catalog: c\nschema: s\nsecret_scope: sc\nsecret_key: k\nvolume_root: {tmp_path}/vol\n")
    monkeypatch.setenv("DBX_SECRET_SC_K", "tok")
    monkeypatch.delenv("HF_TOKEN", raising=False)
    monkeypatch.setenv("DBX_USER", "alice")
    ctx = bootstrap.setup(str(lc), notebook_name="nb1", mlflow_root=str(tmp_path / "mlruns"))
    assert set(ctx.volumes) == set(bootstrap.VOLUMES)
    assert all(os.path.isdir(p) for p in ctx.volumes.values())
    assert ctx.hf_logged_in and os.environ["HF_HOME"] == ctx.hf_home
    assert ctx.experiment_path == "/Users/alice/experiments/nb1" and ctx.experiment_id
    assert ctx.num_workers == 1 and ctx.world_size >= 1
    assert os.environ.get("CUDA_LAUNCH_BLOCKING") != "1"  # never forced (reference perf bug)


# ---------------------------------------------------------------------------------- inference / data
def test_predict_image_and_release():
    torch.manual_seed(0)
    m = nn.Sequential(nn.Flatten(), nn.Linear(3 * 8 * 8, 4))
    img = (np.random.rand(8, 8, 3) * 255).astype(np.uint8)
    pred, p = inference.predict_image(m, img, verbose=False)
    assert 0 <= pred < 4 and 0 < p <= 1
    x = inference.image_to_tensor(img, normalize=False)
    assert x.shape == (1, 3, 8, 8) and float(x.max()) <= 1.0
    assert "allocated" in inference.release_gpu_memory()


def test_tensor_dataset_snapshot(tmp_path):
    ds = SyntheticImages(10, 16, 3, num_classes=5, seed=1)
    path = save_tensor_dataset(ds, str(tmp_path / "train.pt"))
    t = TensorImageDataset(path)
    assert len(t) == 10 and t.images.dtype == torch.uint8
    d = torch.load(path, weights_only=True)  # loads without unpickling arbitrary objects
    assert d["labels"].dtype == torch.int64
    json.dumps({"n": len(t)})
