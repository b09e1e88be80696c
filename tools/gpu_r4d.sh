#!/bin/bash
# round 4: wo weight steps in flight (SLI_WO_NB variant builds) at the K-split default, C1 then C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/ab_variants.sh "base nb3 nb4" --greedy-steps 2 --steps 100 --warmup 20 > gpurun_out/r4d_c1.txt 2>&1 || { cat gpurun_out/r4d_c1.txt; exit 1; }
cat gpurun_out/r4d_c1.txt
bash tools/ab_variants.sh "base nb3 nb4" --greedy-steps 2 --steps 100 --warmup 20 --w-dtype i8 > gpurun_out/r4d_c3.txt 2>&1 || { cat gpurun_out/r4d_c3.txt; exit 1; }
cat gpurun_out/r4d_c3.txt
