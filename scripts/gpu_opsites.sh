cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/op_sites.py > gpurun_out/op_sites_jagged.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --roofline-reps 2 --step-times 1 --steps 30 > gpurun_out/st.json 2>gpurun_out/st.err
