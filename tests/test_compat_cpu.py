"""Compatibility surface with the reference notebooks (CPU, gloo):

* the reference's five DeepSpeed dicts, as literal copies of `02_deepspeed/deepspeed_config.py:5-105`
  (string boolean, "auto" sizes and all), load through ``config.from_deepspeed`` and through a
  2-rank ``DeepspeedTorchDistributor`` run;
* ``frontends.accelerate.Accelerator`` against the installed HF ``accelerate.Accelerator``
  (method / argument names), the notebook's ``train_model(run_id) -> (history, run_id)`` at world 2
  with its MLflow metric and artifact names;
* ``engine.native_module`` inside a real ``torch.nn.parallel.DistributedDataParallel`` wrap;
* per-notebook MLflow model artifact names.
"""
import copy
import inspect
import json
import os

import pytest
import torch
import torch.nn as nn

from dbx_distributed_pytorch_examples_amd import config
from dbx_distributed_pytorch_examples_amd.launch import DeepspeedTorchDistributor, Launcher

pytestmark = pytest.mark.timeout(600)

# ---- literal copies of the reference dicts (02_deepspeed/deepspeed_config.py:5-105) ------------------
_shared = {"gradient_accumulation_steps": 1, "gradient_clipping": 0.3, "per_device_batch_size": 4,
           "learning_rate": 2e-4, "warmup_steps": 100}
REF_BASE = {
    "train_batch_size": "auto",
    "train_micro_batch_size_per_gpu": _shared["per_device_batch_size"],
    "gradient_accumulation_steps": _shared["gradient_accumulation_steps"],
    "gradient_clipping": _shared["gradient_clipping"],
    "bf16": {"enabled": "true"},
    "optimizer": {"type": "AdamW", "params": {"lr": _shared["learning_rate"], "betas": [0.9, 0.999], "eps": 1e-08}},
    "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0, "warmup_max_lr": _shared["learning_rate"],
                                                 "warmup_num_steps": _shared["warmup_steps"],
                                                 "warmup_type": "linear"}},
    "tensorboard": {"enabled": True, "output_path": "/local_disk0/tensorboard", "job_name": "finetune_llama_2_7b"},
    "steps_per_print": 10,
    "wall_clock_breakdown": True,
    "zero_optimization": {},
}
REF_Z1 = copy.deepcopy(REF_BASE)
REF_Z1["zero_optimization"] = {"stage": 1, "overlap_comm": True, "contiguous_gradients": True,
                               "allgather_partitions": True, "allgather_bucket_size": 500000000,
                               "reduce_scatter": True, "reduce_bucket_size": 500000000, "cpu_offload": False}
REF_Z2 = copy.deepcopy(REF_BASE)
REF_Z2["zero_optimization"] = {"stage": 2, "sub_group_size": 1e9, "reduce_bucket_size": "auto"}
REF_Z3 = copy.deepcopy(REF_BASE)
REF_Z3["zero_optimization"] = {"stage": 3, "sub_group_size": 1e9, "reduce_bucket_size": "auto",
                               "stage3_prefetch_bucket_size": "auto", "stage3_param_persistence_threshold": "auto",
                               "stage3_max_live_parameters": 1e7, "stage3_max_reuse_distance": 1e7,
                               "stage3_gather_16bit_weights_on_model_save": True}
REF_Z3_OFF = copy.deepcopy(REF_BASE)
REF_Z3_OFF["zero_optimization"] = {"stage": 3, "offload_optimizer": {"device": "cpu"},
                                   "offload_param": {"device": "cpu"}, "overlap_comm": True,
                                   "contiguous_gradients": True, "sub_group_size": 1e9, "reduce_bucket_size": "auto",
                                   "stage3_prefetch_bucket_size": "auto", "stage3_param_persistence_threshold": "auto",
                                   "stage3_max_live_parameters": 1e7, "stage3_max_reuse_distance": 1e7,
                                   "stage3_gather_16bit_weights_on_model_save": True}
REF_DICTS = {"base": (REF_BASE, 0), "zero_1": (REF_Z1, 1), "zero_2": (REF_Z2, 2), "zero_3": (REF_Z3, 3),
             "zero_3_offload": (REF_Z3_OFF, 3)}


@pytest.mark.parametrize("name", list(REF_DICTS))
def test_reference_deepspeed_dicts_load(name):
    d, stage = REF_DICTS[name]
    cfg = config.from_deepspeed(copy.deepcopy(d), world_size=2, model_numel=11_000_000)
    assert cfg.zero.stage == stage
    assert cfg.optim.name == "adamw" and cfg.optim.lr == 2e-4 and cfg.optim.betas == (0.9, 0.999)
    assert cfg.optim.eps == 1e-8
    assert cfg.optim.weight_decay == 0.0  # DeepSpeed's FusedAdam default (adam_w_mode): the dict omits it
    assert cfg.optim.grad_clip == 0.3 and cfg.precision == "bf16"
    assert cfg.batch_size == 4 and cfg.grad_accum == 1
    assert cfg.sched.name == "warmup_lr" and cfg.sched.warmup_steps == 100 and cfg.sched.warmup_type == "linear"
    assert cfg.log_every == 10 and cfg.wall_clock_breakdown
    assert cfg.tensorboard_dir == "/local_disk0/tensorboard"
    if name == "zero_1":
        assert cfg.zero.reduce_bucket_size == 500_000_000 and not cfg.zero.offload_optimizer
    if name in ("zero_2", "zero_3", "zero_3_offload"):
        assert cfg.zero.reduce_bucket_size == 11_000_000  # "auto": the whole gradient, one bucket
    if name in ("zero_3", "zero_3_offload"):
        assert cfg.zero.stage3_prefetch_bucket_size == int(0.9 * 11_000_000)
        assert cfg.zero.stage3_param_persistence_threshold == 100_000
        assert cfg.zero.stage3_max_live_parameters == 10_000_000
    assert cfg.zero.offload_optimizer == cfg.zero.offload_param == (name == "zero_3_offload")
    # the in-tree dicts are the reference's, key for key
    from dbx_distributed_pytorch_examples_amd.frontends import deepspeed as dsf
    ours = {"base": dsf.deepspeed_base, "zero_1": dsf.deepspeed_zero_1, "zero_2": dsf.deepspeed_zero_2,
            "zero_3": dsf.deepspeed_zero_3, "zero_3_offload": dsf.deepspeed_zero_3_offload}[name]
    assert json.dumps(ours, sort_keys=True) == json.dumps(d, sort_keys=True)


def test_deepspeed_string_booleans_and_batch_checks():
    d = copy.deepcopy(REF_Z1)
    d["bf16"] = {"enabled": "false"}
    assert config.from_deepspeed(d).precision == "fp32"  # a "false" string is false
    d["train_batch_size"] = 32
    with pytest.raises(ValueError, match="train_batch_size"):
        config.from_deepspeed(d, world_size=2)  # 4 x 1 x 2 != 32
    d["train_batch_size"] = 8
    assert config.from_deepspeed(d, world_size=2).batch_size == 4
    del d["train_micro_batch_size_per_gpu"]
    d["train_batch_size"] = 64
    assert config.from_deepspeed(d, world_size=4).batch_size == 16  # micro batch derived
    d["optimizer"] = {"type": "Adam", "params": {"lr": 1e-3}}
    c = config.from_deepspeed(d, config.TrainConfig(), world_size=4)
    assert c.optim.name == "adam" and c.optim.weight_decay == 0.0  # no TrainConfig default leaks in
    d["scheduler"]["params"].pop("warmup_type")
    assert config.from_deepspeed(d, world_size=4).sched.warmup_type == "log"  # DeepSpeed's default


def test_warmup_lr_linear_and_log():
    from dbx_distributed_pytorch_examples_amd.train.schedule import LRSchedule
    lin = LRSchedule("warmup_lr", 2e-4, warmup_steps=100, warmup_type="linear")
    log = LRSchedule("warmup_lr", 2e-4, warmup_steps=100, warmup_type="log")
    assert lin(0) == 0.0 and abs(lin(50) - 1e-4) < 1e-12 and lin(100) == 2e-4 and lin(500) == 2e-4
    import math
    assert abs(log(9) - 2e-4 * math.log(10) / math.log(100)) < 1e-12


def _ds_rank(stage_expected):
    """One rank of a DeepspeedTorchDistributor run: train() picks the DS dict up from the env."""
    from dbx_distributed_pytorch_examples_amd.config import TrainConfig, from_deepspeed
    from dbx_distributed_pytorch_examples_amd.data.datasets import SyntheticImages
    from dbx_distributed_pytorch_examples_amd.models import build_model
    from dbx_distributed_pytorch_examples_amd.train.engine import train
    ds = json.loads(os.environ["DBX_DEEPSPEED_CONFIG"])
    cfg = TrainConfig(model="resnet18", num_classes=10, max_steps=2, log_every=0)
    cfg.data.num_workers = 0
    seen = from_deepspeed(ds, cfg)  # what train() applies (world from the launcher's env)
    torch.manual_seed(0)
    tr = SyntheticImages(16, 32, 3, 10, seed=1)
    res = train(cfg, model=build_model("resnet18", num_classes=10), train_dataset=tr, log_mlflow=False)
    return (seen.zero.stage, seen.optim.name, seen.optim.lr, seen.optim.grad_clip, seen.precision, seen.batch_size,
            res.steps, res.engine, int(os.environ["WORLD_SIZE"]))


@pytest.mark.parametrize("name", ["zero_1", "zero_2", "zero_3", "zero_3_offload"])
def test_reference_deepspeed_dicts_two_rank_run(name):
    d, stage = REF_DICTS[name]
    out = DeepspeedTorchDistributor(numGpus=2, nnodes=1, localMode=True, useGpu=False,
                                    deepspeedConfig=copy.deepcopy(d)).run(_ds_rank, stage)
    assert out == (stage, "adamw", 2e-4, 0.3, "bf16", 4, 2, "autograd", 2), out


def test_zero3_persistence_and_prefetch_knobs():
    """stage3_param_persistence_threshold keeps small units gathered; prefetch issues the next
    units' gathers ahead (world 1: the knobs are accepted, the persistent unit stays materialised
    across an optimizer step)."""
    from dbx_distributed_pytorch_examples_amd.models import build_model
    from dbx_distributed_pytorch_examples_amd.parallel.fsdp import ShardedDataParallel
    o = config.OptimizerConfig(name="adamw", lr=1e-3)
    m = build_model("resnet18", num_classes=10)
    sdp = ShardedDataParallel(m, o, persistence_threshold=100_000, prefetch_elems=5_000_000)
    pers = [u for u in sdp.units if u.persistent]
    assert pers and all(u.n < 100_000 for u in pers) and all(u.gathered for u in pers)
    x, y = torch.randn(2, 3, 32, 32), torch.randint(0, 10, (2,))
    nn.functional.cross_entropy(sdp(x), y).backward()
    sdp.finish_gradient_sync()
    sdp.optimizer_step()
    assert all(u.gathered for u in pers)
    assert not any(u.gathered for u in sdp.units if not u.persistent)


# ---- Accelerate -------------------------------------------------------------------------------------
_FACADE_METHODS = ["prepare", "autocast", "backward", "gather", "gather_for_metrics", "reduce", "wait_for_everyone",
                   "unwrap_model", "init_trackers", "log", "end_training", "save", "no_sync", "print",
                   "clip_grad_norm_", "main_process_first", "local_main_process_first", "free_memory", "accumulate",
                   "save_state", "load_state", "get_state_dict", "split_between_processes", "pad_across_processes",
                   "set_trigger", "check_trigger"]
_FACADE_PROPS = ["num_processes", "process_index", "local_process_index", "is_main_process", "is_local_main_process",
                 "device", "mixed_precision", "distributed_type", "use_distributed", "sync_gradients",
                 "is_last_process"]


def test_accelerator_facade_matches_hf_accelerate():
    hf = pytest.importorskip("accelerate")
    from dbx_distributed_pytorch_examples_amd.frontends.accelerate import Accelerator
    for name in _FACADE_PROPS:
        assert isinstance(inspect.getattr_static(hf.Accelerator, name), property), name
        assert isinstance(inspect.getattr_static(Accelerator, name), property), name
    for name in _FACADE_METHODS:
        theirs, ours = getattr(hf.Accelerator, name), getattr(Accelerator, name)
        try:
            tp = inspect.signature(inspect.unwrap(theirs)).parameters
        except (TypeError, ValueError):
            continue
        if any(p.kind == p.VAR_POSITIONAL for p in tp.values()) and len(tp) <= 2:
            continue  # (*args, **kwargs) decorators (log / init_trackers): names checked below by call
        op = inspect.signature(ours).parameters
        # every argument of the HF method is accepted under the same name (positional order kept)
        tnames = [n for n, p in tp.items() if p.kind in (p.POSITIONAL_OR_KEYWORD, p.KEYWORD_ONLY)]
        onames = [n for n, p in op.items() if p.kind in (p.POSITIONAL_OR_KEYWORD, p.KEYWORD_ONLY)]
        assert onames[:len(tnames)] == tnames or set(tnames) <= set(onames), (name, tnames, onames)
    # the (*args, **kwargs)-decorated ones: the documented argument names
    assert list(inspect.signature(Accelerator.log).parameters)[:3] == ["self", "values", "step"]
    assert list(inspect.signature(Accelerator.init_trackers).parameters)[:3] == ["self", "project_name", "config"]
    for name in ("gradient_accumulation_steps", "mixed_precision", "cpu", "log_with", "split_batches",
                 "device_placement"):
        assert name in inspect.signature(hf.Accelerator.__init__).parameters
        assert name in inspect.signature(Accelerator.__init__).parameters


def _train_model_rank(root):
    os.environ["DBX_MLRUNS"] = root
    from torch.utils.data import DataLoader
    from dbx_distributed_pytorch_examples_amd.data.datasets import SyntheticImages
    from dbx_distributed_pytorch_examples_amd.frontends.accelerate import Accelerator, train_model
    from dbx_distributed_pytorch_examples_amd.parallel.sampler import ShardSampler
    acc = Accelerator(cpu=True, log_with="mlflow")
    torch.manual_seed(0)
    import numpy as np

    def tf(img):
        return torch.from_numpy(np.array(img)).permute(2, 0, 1).float() / 255
    tr = SyntheticImages(16, 16, 3, 4, seed=1, transform=tf)
    te = SyntheticImages(8, 16, 3, 4, seed=2, transform=tf)
    model = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.ReLU(), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(8, 4))
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=2)
    cfg = {"batch_size": 4, "num_epochs": 2, "learning_rate": 1e-3, "weight_decay": 0.0, "num_classes": 4,
           "save_every": 1}
    model, opt, trl, tel = acc.prepare(model, opt, DataLoader(tr, batch_size=4, sampler=ShardSampler(tr)),
                                       DataLoader(te, batch_size=4, sampler=ShardSampler(te, shuffle=False)))
    history, run_id = train_model(None, accelerator=acc, model=model, optimizer=opt, scheduler=sched,
                                  criterion=nn.CrossEntropyLoss(), train_loader=trl, test_loader=tel, config=cfg)
    return acc.process_index, history, run_id


def test_accelerate_train_model_two_ranks(tmp_path):
    root = str(tmp_path / "mlruns")
    out = Launcher(2, use_gpu=False).run(_train_model_rank, root)
    rank, history, run_id = out
    assert rank == 0 and run_id
    assert set(history) == {"train_loss", "train_acc", "test_loss", "test_acc", "lr"} and len(history["lr"]) == 2
    run_dir = [os.path.join(root, e, run_id) for e in os.listdir(root) if os.path.isdir(os.path.join(root, e, run_id))]
    assert run_dir
    metrics = set(os.listdir(os.path.join(run_dir[0], "metrics")))
    assert {"train_loss", "train_accuracy", "test_loss", "test_accuracy", "learning_rate"} <= metrics
    arts = set(os.listdir(os.path.join(run_dir[0], "artifacts")))
    assert {"training_history.json", "best_model", "checkpoints"} <= arts, arts


def _run_id_ranks(root):
    os.environ["DBX_MLRUNS"] = root
    from dbx_distributed_pytorch_examples_amd.frontends.accelerate import Accelerator, broadcast_run_id
    from dbx_distributed_pytorch_examples_amd.utils import mlflow_compat as mlflow
    acc = Accelerator(cpu=True)
    rid = mlflow.start_run().info.run_id if acc.is_main_process else None
    got = broadcast_run_id(rid, acc)
    import torch.distributed as tdist
    both = [None, None]
    tdist.all_gather_object(both, got)
    return both


def test_run_id_broadcast_two_ranks(tmp_path):
    a, b = Launcher(2, use_gpu=False).run(_run_id_ranks, str(tmp_path / "mlruns"))
    assert a == b and a


def _torch_ddp_native(_):
    """engine.native_module wrapped by torch's own DDP (what the real HF Accelerator.prepare does at
    world > 1): the wrapper is made inert, the module's own all-reduce averages the gradient, and
    a second iteration runs (torch DDP would otherwise raise on the unfinished reduction)."""
    import warnings
    import torch.distributed as tdist
    from torch.nn.parallel import DistributedDataParallel as TorchDDP
    from dbx_distributed_pytorch_examples_amd.engine.native_module import native_module
    from dbx_distributed_pytorch_examples_amd.models import build_model
    from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist
    ddist.init_distributed(device="cpu")
    torch.manual_seed(0)
    nm = native_module(build_model("resnet18", num_classes=10), 4, (32, 32), torch.device("cpu")).train()
    w = TorchDDP(nm)
    opt = torch.optim.SGD(nm.parameters(), lr=0.05)
    rank = tdist.get_rank()
    ok = []
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        for it in range(2):
            g = torch.Generator().manual_seed(10 * it + rank)
            x, y = torch.randn(4, 3, 32, 32, generator=g), torch.randint(0, 10, (4,), generator=g)
            opt.zero_grad()
            nn.functional.cross_entropy(w(x), y).backward()
            grad = torch.cat([p.grad.reshape(-1) for p in nm.parameters()])
            both = [torch.empty_like(grad) for _ in range(2)]
            tdist.all_gather(both, grad)
            ok.append(torch.equal(both[0], both[1]) and float(grad.norm()) > 0)
            opt.step()
    inert = any("inert" in str(c.message) for c in caught)
    ddist.destroy()
    return ok, inert


def test_native_module_under_torch_ddp_two_ranks():
    ok, inert = Launcher(2, use_gpu=False).run(_torch_ddp_native, None)
    assert ok == [True, True] and inert


def test_train_func_logs_reference_artifact_names(tmp_path, monkeypatch):
    """TD / DS train_funcs log the model under the notebooks' artifact names."""
    monkeypatch.setenv("DBX_MLRUNS", str(tmp_path / "mlruns"))
    monkeypatch.setenv("DBX_FORCE_CPU", "1")
    from dbx_distributed_pytorch_examples_amd.data.datasets import SyntheticImages
    from dbx_distributed_pytorch_examples_amd.frontends import deepspeed as dsf
    from dbx_distributed_pytorch_examples_amd.frontends import torch_distributor as td
    from dbx_distributed_pytorch_examples_amd.utils import mlflow_compat as mlflow
    tr, te = SyntheticImages(8, 32, 3, 10, seed=1), SyntheticImages(4, 32, 3, 10, seed=2)
    td.train_func(train_dataset=tr, test_dataset=te, batch_size=4, epochs=1, mlflow_run_id="x")
    dsf.train_func(train_dataset=tr, test_dataset=te, batch_size=4, num_epochs=1, mlflow_parent_run="x",
                   model_name=dsf.MODEL_NAMES["tiny_imagenet"])
    root = str(tmp_path / "mlruns")
    names = set()
    for e in os.listdir(root):
        ed = os.path.join(root, e)
        for r in (os.listdir(ed) if os.path.isdir(ed) else []):
            a = os.path.join(ed, r, "artifacts")
            if os.path.isdir(a):
                names |= set(os.listdir(a))
    assert {"cifar_torch_distributor_resnet", "tiny_imagenet_torch_distributor_resnet"} <= names, names
    assert mlflow.active_run() is None


def test_native_module_fallback_grads_follow_param_layout():
    """native_module's torch-module path (a batch of another shape): the weight gradient of the conv
    backward arrives in its own layout (contiguous from MIOpen) while the parameters are channels-last
    views of the program's KRSC master; the wrapper's hooks hand autograd channels-last gradients for
    channels-last parameters, and leave every other gradient untouched. (On the GPU the Composer test
    in test_program_gpu.py must run without the layout-contract warning.)"""
    from dbx_distributed_pytorch_examples_amd.engine.native_module import _grad_to_param_layout, native_module
    from dbx_distributed_pytorch_examples_amd.models import build_model
    r18 = build_model("resnet18", num_classes=10)
    native_module(r18, batch=None, device=torch.device("cpu"))
    assert all(p._backward_hooks for p in r18.parameters() if p.dim() == 4)
    w_cl = torch.randn(8, 3, 3, 3).contiguous(memory_format=torch.channels_last)
    g = torch.randn(8, 3, 3, 3)
    out = _grad_to_param_layout(w_cl)(g)
    assert out.is_contiguous(memory_format=torch.channels_last) and torch.equal(out, g)
    w_c = torch.randn(8, 3, 3, 3)
    assert _grad_to_param_layout(w_c)(g) is g  # contiguous parameter: nothing to do
    w_1 = torch.randn(8, 1, 1, 1)  # both layouts at once (1x1 / 1-channel): nothing to do
    assert _grad_to_param_layout(w_1)(g[:, :1, :1, :1]).data_ptr() == g.data_ptr()


def test_repoint_keeps_a_precompile_grad_in_the_new_layout():
    """A gradient that exists before the program is compiled (a first batch through the torch module)
    is re-laid-out with the parameter (KRSC master view: channels-last), values kept."""
    from dbx_distributed_pytorch_examples_amd.engine.program import _repoint
    p = torch.nn.Parameter(torch.randn(8, 4, 3, 3))
    p.grad = torch.randn(8, 4, 3, 3)
    g0 = p.grad.clone()
    master = torch.empty(8 * 3 * 3 * 4)
    view = master.view(8, 3, 3, 4).permute(0, 3, 1, 2)
    _repoint(p, view)
    assert p.grad.stride() == view.stride() and torch.equal(p.grad, g0)


def test_flat_grad_views_follow_channels_last_params():
    """The DDP flat gradient buffer views channels-last conv weights with their own strides (the
    GPU AutogradTrainer runs the model channels-last): autograd accumulates in place without the
    layout-contract warning, gradients match a plain model's; ZeRO over the flat buffer keeps the
    master in the same memory order (one step equals torch Adam's)."""
    import warnings
    from dbx_distributed_pytorch_examples_amd.engine.autograd_trainer import AutogradTrainer
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import OptimConfig
    from dbx_distributed_pytorch_examples_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3, padding=1), torch.nn.ReLU(), torch.nn.Conv2d(8, 6, 3),
                              torch.nn.AdaptiveAvgPool2d(1), torch.nn.Flatten(), torch.nn.Linear(6, 4))
    ref = copy.deepcopy(net)
    net = net.to(memory_format=torch.channels_last)
    ddp = DistributedDataParallel(net)
    x = torch.randn(5, 3, 9, 9)
    for _ in range(2):
        with warnings.catch_warnings():
            warnings.simplefilter("error")
            ddp(x.contiguous(memory_format=torch.channels_last)).square().sum().backward()
        ref(x).square().sum().backward()
    buf = ddp.flat.buffer
    for p, q in zip(net.parameters(), ref.parameters()):
        assert p.grad.stride() == p.stride() and buf.data_ptr() <= p.grad.data_ptr() < buf.data_ptr() + 4 * buf.numel()
        assert torch.allclose(p.grad, q.grad, atol=1e-5, rtol=1e-4)
    m1 = copy.deepcopy(ref).to(memory_format=torch.channels_last)
    m2 = copy.deepcopy(ref)
    o = OptimConfig(name="adam", lr=1e-2, weight_decay=0.0)
    tr = AutogradTrainer(m1, torch.device("cpu"), o, zero_stage=1, channels_last=False)
    opt = torch.optim.Adam(m2.parameters(), lr=1e-2)
    y = torch.randint(0, 4, (5,))
    tr.step(x.contiguous(memory_format=torch.channels_last), y)
    torch.nn.functional.cross_entropy(m2(x), y).backward()
    opt.step()
    for p, q in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=1e-5, rtol=1e-4)
