#!/bin/bash
# Round-4 end-of-round evidence on one GPU box -> gpurun_out/TAG/: tools/final_session.sh (full
# GPU suite, smoke, the default bench line, rocprofv3 kernel stats of the same command + per-
# kernel medians, FETCH/WRITE traffic stamped with the kernel-source digest), then the SQ
# counter passes of the fused kernel (tools/pmc_fused.sh: k_fused4 at B = 32).
set -o pipefail
TAG=${1:-r04final}
bash tools/final_session.sh "$TAG" || exit 1
bash tools/pmc_fused.sh "$TAG/sq" fused 32 || exit 1
