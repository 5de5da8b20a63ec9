#!/bin/bash
# Final round-6 library: smoke + the whole -m gpu suite, the default bench line and the c4
# line (scripts/gpu_final2.sh), then a kernel trace of the default bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/gpu_final2.sh; rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
mkdir -p gpurun_out/fin3
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/fin3/prof" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 3 \
  > "$GRAFT_REPO_ROOT/gpurun_out/fin3/prof.log" 2>&1
echo "trace rc=$?"
