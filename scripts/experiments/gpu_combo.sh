#!/bin/bash
# gradient diagnostic table; the new link / PAIRPRE and ring tests on the default library;
# the encoder layer-0 slot variant (tests + A/B); A/B of the per-node link first layer
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python scripts/grad_diag.py > gpurun_out/grad_diag.log 2>&1
rc=$?; echo "grad_diag rc=$rc"; tail -10 gpurun_out/grad_diag.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f32.py tests/test_gpu_parity.py tests/test_gpu_blocks.py "tests/test_distributed.py::test_rccl_collectives_on_device" > gpurun_out/combo_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAIL|Error" gpurun_out/combo_tests.log | head; tail -2 gpurun_out/combo_tests.log
if [ $rc -ge 124 ]; then exit $rc; fi
bash scripts/gpu_k0slot.sh; rc=$?
if [ $rc -ge 124 ]; then exit $rc; fi
AB="linkpre:RG_LINK_PRE=1;linkpair:RG_LINK_PRE=0" ROUNDS=2 bash scripts/gpu_ab.sh
