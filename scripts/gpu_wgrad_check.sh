# wgrad: parity tests, the microbench at the bench's shapes, a bench line + step breakdown.
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_wgrad.py tests/test_gpu_model.py > gpurun_out/wgrad_test.log 2>&1
timeout -k 10 200 python -u scripts/microbench/wgrad.py > gpurun_out/wgrad_micro.txt 2>&1
timeout -k 10 300 python -u bench.py --cpu-baseline 0 > gpurun_out/wgrad_bench.json 2> gpurun_out/wgrad_bench.err
rm -rf /tmp/kw && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kw -o run -- python bench.py --steps 10 --warmup 5 --cpu-baseline 0 --roofline-reps 1 > gpurun_out/wgrad_kt.log 2>&1
python scripts/step_breakdown.py $(find /tmp/kw -name "*kernel_trace.csv" | head -n 1) k_seq_ranges 5 > gpurun_out/wgrad_step_breakdown.txt
