#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/debug_trajectory.py cuda > gpurun_out/traj.log 2>&1; echo "traj rc=$?"; cat gpurun_out/traj.log | tail -9
timeout -k 10 200 python tools/debug_grads.py cuda resnet18 32 32 > gpurun_out/grads.log 2>&1; echo "grads rc=$?"; cat gpurun_out/grads.log | tail -70
