#!/bin/bash
# round 4 final: the whole -m gpu suite + smoke + the C2 bench with its trace / PMC, then the C2 variant A/B
set -e
cd "$(dirname "$0")/.."
bash tools/gpu_r04_full.sh r04g
bash tools/gpu_r04_c2v.sh
echo all done
