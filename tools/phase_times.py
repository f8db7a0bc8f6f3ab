"""Per-phase device time of the native ResNet-50 step (DBX_PROFILE=phases: eager phases with
hipEvent timers and roctx ranges)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models import build_model  # noqa: E402

B = int(os.environ.get("BATCH", 1024))
tr = NativeTrainer(build_model("resnet50"), B, (224, 224), torch.device("cuda"), optim=OptimConfig())
tr.prog.img_u8.copy_(torch.randint(0, 256, tr.prog.img_u8.shape, dtype=torch.uint8))
tr.prog.labels.copy_(torch.randint(0, 1000, (B,)))
for _ in range(3):
    tr.step()
tr.phase_timer.reset()
for _ in range(5):
    tr.step()
s = tr.phase_timer.summary()
tot = sum(v["mean_ms"] for v in s.values())
print(json.dumps({k: round(v["mean_ms"], 3) for k, v in s.items()}))
print(f"sum of phases {tot:.2f} ms at batch {B} (eager launches)")
