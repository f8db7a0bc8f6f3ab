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

# ---- config dicts: key for key and value for value the reference's (`02_deepspeed/deepspeed_config.py:5-105`,
# including its string boolean "true" and the "auto" sizes, which config.from_deepspeed resolves) ----------
shared_parameters: Dict[str, Any] = {
    "gradient_accumulation_steps": 1,
    "gradient_clipping": 0.3,
    "per_device_batch_size": 4,
    "learning_rate": 2e-4,
    "warmup_steps": 100,
}

deepspeed_base: Dict[str, Any] = {
    "train_batch_size": "auto",
    "train_micro_batch_size_per_gpu": shared_parameters["per_device_batch_size"],
    "gradient_accumulation_steps": shared_parameters["gradient_accumulation_steps"],
    "gradient_clipping": shared_parameters["gradient_clipping"],
    "bf16": {"enabled": "true"},
    "optimizer": {"type": "AdamW",
                  "params": {"lr": shared_parameters["learning_rate"], "betas": [0.9, 0.999], "eps": 1e-08}},
    "scheduler": {"type": "WarmupLR",
                  "params": {"warmup_min_lr": 0, "warmup_max_lr": shared_parameters["learning_rate"],
                             "warmup_num_steps": shared_parameters["warmup_steps"], "warmup_type": "linear"}},
    "tensorboard": {"enabled": True, "output_path": "/local_disk0/tensorboard", "job_name": "finetune_llama_2_7b"},
    "steps_per_print": 10,
    "wall_clock_breakdown": True,
    "zero_optimization": {},
}


def _with_zero(zero: Dict[str, Any]) -> Dict[str, Any]:
    c = copy.deepcopy(deepspeed_base)
    c["zero_optimization"] = zero
    return c


deepspeed_zero_1 = _with_zero({"stage": 1, "overlap_comm": True, "contiguous_gradients": True,
                               "allgather_partitions": True, "allgather_bucket_size": 500000000,
                               "reduce_scatter": True, "reduce_bucket_size": 500000000, "cpu_offload": False})
deepspeed_zero_2 = _with_zero({"stage": 2, "sub_group_size": 1e9, "reduce_bucket_size": "auto"})
_stage3 = {"sub_group_size": 1e9, "reduce_bucket_size": "auto", "stage3_prefetch_bucket_size": "auto",
           "stage3_param_persistence_threshold": "auto", "stage3_max_live_parameters": 1e7,
           "stage3_max_reuse_distance": 1e7, "stage3_gather_16bit_weights_on_model_save": True}
deepspeed_zero_3 = _with_zero({"stage": 3, **_stage3})
deepspeed_zero_3_offload = _with_zero({"stage": 3, "offload_optimizer": {"device": "cpu"},
                                       "offload_param": {"device": "cpu"}, "overlap_comm": True,
                                       "contiguous_gradients": True, **_stage3})

# short aliases used by the examples / tests
base_config = deepspeed_base
zero_1, zero_2, zero_3, zero_3_offload = deepspeed_zero_1, deepspeed_zero_2, deepspeed_zero_3, deepspeed_zero_3_offload
deepspeed_config = zero_1

# MLflow model artifact names of the DS notebooks
MODEL_NAMES = {"cifar": "deepspeed_cifar_model",                            # 01_cifar_deepspeed_resnet.py:269
               "tiny_imagenet": "tiny_imagenet_torch_distributor_resnet",   # 02_tiny_imagenet_deepspeed_resnet.py:301
               "imagenet_1k": "deepspeed_cifar_model"}                      # 03_1k_imagenet_deepspeed_resnet.py:249


def train_func(*, train_dataset, test_dataset, batch_size: int = 128, num_epochs: int = 1,
               mlflow_parent_run=None, patience: Optional[int] = None, deepspeed_config: Optional[dict] = None,
               arch: str = "resnet18", frozen_backbone: bool = True, learning_rate: float = 1e-5,
               model_name: str = MODEL_NAMES["cifar"], **_):
    """DS-notebook train_func: Adam(lr=1e-5) by default; with ``deepspeed_config`` the DS dict wins
    (its "auto" entries resolved against this model and the launched world size). The trained model
    is logged to MLflow as ``model_name``."""
    num_classes = getattr(test_dataset, "num_classes", None) or getattr(train_dataset, "num_classes", 10)
    model = FrozenBackboneClassifier(arch, num_classes) if frozen_backbone else build_model(arch, num_classes=num_classes)
    cfg = TrainConfig(model=arch, num_classes=num_classes, batch_size=batch_size, epochs=num_epochs,
                      patience=patience or 0, experiment=os.environ.get("MLFLOW_EXPERIMENT_NAME", "deepspeed"),
                      model_name=model_name)
    cfg.optim.name, cfg.optim.lr, cfg.optim.weight_decay = "adam", learning_rate, 0.0
    if deepspeed_config is not None:
        cfg = from_deepspeed(deepspeed_config, cfg, model_numel=sum(p.numel() for p in model.parameters()))
        cfg.batch_size = batch_size  # the notebook passes its own per-GPU batch explicitly
    res = _train(cfg, model=model, train_dataset=train_dataset, eval_dataset=test_dataset,
                 log_mlflow=mlflow_parent_run is not None)
    return res.model
