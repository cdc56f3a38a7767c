# Occurrence sort: parity tests, the embedding / model tests that run it, a bench line and a step breakdown.
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread ${TESTS:-tests/test_gpu_embedding.py tests/test_gpu_model.py tests/test_gpu_sharding.py} > gpurun_out/sort_test.log 2>&1
timeout -k 10 300 python -u bench.py --cpu-baseline 0 > gpurun_out/sort_bench.json 2> gpurun_out/sort_bench.err
rm -rf /tmp/ks && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/ks -o run -- python bench.py --steps 10 --warmup 5 --cpu-baseline 0 --roofline-reps 1 > gpurun_out/sort_kt.log 2>&1
python scripts/step_breakdown.py $(find /tmp/ks -name "*kernel_trace.csv" | head -n 1) k_seq_ranges 5 > gpurun_out/sort_step_breakdown.txt
