#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes (HBM bytes, instruction mix, stalls) of bench.py.
# Only the summaries stay under gpurun_out/ (the raw per-dispatch traces are deleted: gpurun merges
# at most 64 MiB back).
set -u
TAG=${TAG:-r01}
ARGS=${ARGS:-"--steps 30 --warmup 3 --no-cpu-baseline --rollout-T 0 --c2-envs 0 --c5-envs 0"}
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { timeout -k 10 400 rocprofv3 "$@" -- python bench.py $ARGS > /dev/null 2>&1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o trace --output-format csv -- python bench.py $ARGS > gpurun_out/prof_${TAG}_bench.log 2>&1 || exit $?
find gpurun_out/prof_$TAG -name '*kernel_stats.csv' -exec cp {} gpurun_out/kernel_stats_$TAG.csv \;
python3 scripts/trace_by_grid.py gpurun_out/prof_$TAG gpurun_out/kernel_stats_by_grid_$TAG.csv || exit $?
run --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o pmc --output-format csv || exit $?
run --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o pmc --output-format csv || exit $?
run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_sq_$TAG -o pmc --output-format csv || exit $?
run --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU -d gpurun_out/pmc_sq2_$TAG -o pmc --output-format csv || exit $?
run --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_grbm_$TAG -o pmc --output-format csv || exit $?
python3 scripts/pmc_summary.py $TAG ${WORKLOAD:-8x64x5x32768} > gpurun_out/pmc_summary_$TAG.txt || exit $?
rm -rf gpurun_out/prof_$TAG gpurun_out/pmc_*_$TAG
cat gpurun_out/kernel_stats_$TAG.csv
echo done
