#!/bin/bash
# Round-6 validation (scripts/gpu_r06.sh) then an interleaved A/B of the fused node phase
# (default library) against the two-launch layer (lib/variants/libradargnn_nofuse.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/gpu_r06.sh; rc=$?
if [ $rc -ge 124 ]; then exit $rc; fi
AB="base:;lib_nofuse:" ROUNDS=2 bash scripts/gpu_ab.sh; rc2=$?
exit $(( rc > rc2 ? rc : rc2 ))
