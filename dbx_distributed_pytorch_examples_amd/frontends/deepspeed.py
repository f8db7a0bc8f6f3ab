"""DeepSpeed-style configs and ``train_func`` (`02_deepspeed/*.py`) — with the config APPLIED.

The reference builds DeepSpeed dicts (`02_deepspeed/deepspeed_config.py`: bf16, AdamW 2e-4,
WarmupLR over 100 steps, gradient clipping 0.3, micro-batch 4, ZeRO-1/2/3/3-offload) but never
passes them (`01_cifar_deepspeed_resnet.py:108` is commented out) and never calls
``deepspeed.initialize``. Here ``train_func(..., deepspeed_config=zero_1)`` (or a
``DeepspeedTorchDistributor(deepspeedConfig=...)``) maps the dict onto the engine: bf16 compute,
AdamW/SGD, WarmupLR, global-norm clipping, ZeRO stage 1/2 sharded optimizer state
(``parallel.zero``) and stage 3 parameter sharding with optional CPU offload of the optimizer /
parameters (``parallel.fsdp``, autograd engine).
"""
from __future__ import annotations

import copy
import os
from typing import Any, Dict, Optional

from ..config import TrainConfig, from_deepspeed
from ..launch import DeepspeedTorchDistributor  # noqa: F401  (re-export)
from ..models import FrozenBackboneClassifier, build_model
from ..train.engine import train as _train

# ---- config dicts (same keys / values as the reference's deepspeed_config.py) -------------------
base_config: Dict[str, Any] = {
    "bf16": {"enabled": True},
    "optimizer": {"type": "AdamW", "params": {"lr": 2e-4, "betas": [0.9, 0.999], "eps": 1e-8, "weight_decay": 0.01}},
    "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0, "warmup_max_lr": 2e-4, "warmup_num_steps": 100}},
    "gradient_clipping": 0.3,
    "train_micro_batch_size_per_gpu": 4,
    "gradient_accumulation_steps": 1,
    "steps_per_print": 100,
    "wall_clock_breakdown": True,
    "tensorboard": {"enabled": True, "output_path": "/tmp/tensorboard", "job_name": "dbx"},
}


def _with_zero(stage: int, **zero) -> Dict[str, Any]:
    c = copy.deepcopy(base_config)
    c["zero_optimization"] = {"stage": stage, **zero}
    return c


zero_1 = _with_zero(1, overlap_comm=True, contiguous_gradients=True, reduce_scatter=True,
                    reduce_bucket_size=5e8, allgather_bucket_size=5e8)
zero_2 = _with_zero(2, overlap_comm=True, contiguous_gradients=True, reduce_scatter=True,
                    reduce_bucket_size=5e8, allgather_bucket_size=5e8)
zero_3 = _with_zero(3, overlap_comm=True, contiguous_gradients=True, sub_group_size=1e9,
                    stage3_prefetch_bucket_size=5e8, stage3_param_persistence_threshold=1e6)
zero_3_offload = _with_zero(3, offload_optimizer={"device": "cpu", "pin_memory": True},
                            offload_param={"device": "cpu", "pin_memory": True})
deepspeed_config = zero_1

# the reference module's names (`02_deepspeed/deepspeed_config.py:5-105`)
shared_parameters = {"gradient_accumulation_steps": 1, "gradient_clipping": 0.3, "per_device_batch_size": 4,
                     "learning_rate": 2e-4, "warmup_steps": 100}
deepspeed_base = base_config
deepspeed_zero_1, deepspeed_zero_2, deepspeed_zero_3, deepspeed_zero_3_offload = zero_1, zero_2, zero_3, zero_3_offload


def train_func(*, train_dataset, test_dataset, batch_size: int = 128, num_epochs: int = 1,
               mlflow_parent_run=None, patience: Optional[int] = None, deepspeed_config: Optional[dict] = None,
               arch: str = "resnet18", frozen_backbone: bool = True, learning_rate: float = 1e-5, **_):
    """DS-notebook train_func: Adam(lr=1e-5) by default; with ``deepspeed_config`` the DS dict wins."""
    num_classes = getattr(test_dataset, "num_classes", None) or getattr(train_dataset, "num_classes", 10)
    model = FrozenBackboneClassifier(arch, num_classes) if frozen_backbone else build_model(arch, num_classes=num_classes)
    cfg = TrainConfig(model=arch, num_classes=num_classes, batch_size=batch_size, epochs=num_epochs,
                      patience=patience or 0, experiment=os.environ.get("MLFLOW_EXPERIMENT_NAME", "deepspeed"))
    cfg.optim.name, cfg.optim.lr, cfg.optim.weight_decay = "adam", learning_rate, 0.0
    if deepspeed_config is not None:
        cfg = from_deepspeed(deepspeed_config, cfg)
        cfg.batch_size = batch_size  # the notebook passes its own per-GPU batch explicitly
    res = _train(cfg, model=model, train_dataset=train_dataset, eval_dataset=test_dataset,
                 log_mlflow=mlflow_parent_run is not None)
    return res.model
