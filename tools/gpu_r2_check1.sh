set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_lars.py tests/test_program_gpu.py -k "lr_schedule or lars or baseline_config" > gpurun_out/t_new.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/t_new.log; exit 1; }
tail -3 gpurun_out/t_new.log
timeout -k 10 200 python tools/determinism_check.py --optim lars --steps 5 && timeout -k 10 200 python tools/determinism_check.py --optim adamw --steps 5
bash tools/gpu_pmc_step.sh 1024
