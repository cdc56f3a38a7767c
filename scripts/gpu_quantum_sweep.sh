cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for q in 4096 1024 512; do
  timeout -k 10 300 python -u bench.py --cpu-baseline 0 --roofline-reps 2 --jagged-quantum $q > gpurun_out/q$q.json 2>gpurun_out/q$q.err || exit 1
done
