#!/bin/bash
# Round-3 end-of-round evidence on one GPU box -> gpurun_out/TAG/: tools/final_session.sh (full
# GPU suite, smoke, the default bench line, rocprofv3 kernel stats of the same command + per-
# kernel medians, FETCH/WRITE traffic stamped with the kernel-source digest), then the SQ
# counter passes of the fused kernel (tools/pmc_fused.sh).
set -o pipefail
TAG=${1:-r03final}
bash tools/final_session.sh "$TAG" || exit 1
bash tools/pmc_fused.sh "$TAG/sq" fused 32 || exit 1
