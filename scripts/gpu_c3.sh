set -e -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharding.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/shard_test.log 2>&1
timeout -k 10 500 python -u bench.py --cpu-baseline 0 --sharded 1 --items 20000000 --steps 10 --warmup 4 --roofline-reps 5 > gpurun_out/c3w1_bench.json 2> gpurun_out/c3w1_bench.err
