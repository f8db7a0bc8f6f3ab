set -o pipefail
mkdir -p gpurun_out
cp dbx_distributed_pytorch_examples_amd/ops/tune_table.json gpurun_out/tune_tmp.json
timeout -k 10 400 python tools/tune_conv.py --modes wgrad --batch 1024 --verbose --out gpurun_out/tune_tmp.json > gpurun_out/tune_wgrad_all.log 2>&1 || { echo "tune FAILED"; tail -20 gpurun_out/tune_wgrad_all.log; exit 1; }
grep "^  wgrad" gpurun_out/tune_wgrad_all.log
