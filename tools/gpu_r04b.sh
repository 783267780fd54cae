#!/bin/bash
# Round-4 roofline evidence for configs 3 and 5 at HEAD (GPU box): PMC passes (tools/pmc_configs.sh), kernel stats of
# the forward configs and of the gradient configs, and the gradient timings.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CFGS=3 bash tools/pmc_configs.sh || exit $?
CFGS=5 bash tools/pmc_configs.sh || exit $?
CFGS=3,5 bash tools/gpu_session.sh profcfg gradcfg || exit $?
CFGS=3,5 bash tools/gpu_session.sh profgrad || exit $?
echo r04b done
