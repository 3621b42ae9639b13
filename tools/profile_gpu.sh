#!/bin/bash
# Profiles bench.py's headline workload on the GPU box: one kernel-trace/stats pass, then separate PMC
# passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; SQ counters in their own pass).
# Usage (from the repo root on the box): tools/profile_gpu.sh [workload] [tag]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
W=${1:-odt}
TAG=${2:-r02}
OUT=$R/gpurun_out/prof_${W}_${TAG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --workload $W --no-side --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $BENCH --steps 3 --warmup 1 > $OUT/bench_under_kt.json
# PMC passes: one untimed step first, so the two counted steps run the steady-state launch size (prof_summary.py counts
# the last two steps' dispatches only); the HBM passes also count SQ_WAVES, so a dispatch whose waves were context-saved and
# restored (SQ_WAVES above its grid's waves: the save writes every resident wave's VGPRs/SGPRs and the CUs' LDS,
# DESIGN.md section 6, round 5) can be told apart from the kernel's own traffic
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE SQ_WAVES --kernel-trace -d $OUT/fetch -o fetch --output-format csv -- python3 $BENCH --steps 2 --warmup 1 > /dev/null
timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE SQ_WAVES --kernel-trace -d $OUT/write -o write --output-format csv -- python3 $BENCH --steps 2 --warmup 1 > /dev/null
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/sq -o sq --output-format csv -- python3 $BENCH --steps 2 --warmup 1 > /dev/null
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/lds -o lds --output-format csv -- python3 $BENCH --steps 2 --warmup 1 > /dev/null
python3 $R/tools/prof_summary.py $OUT $R/gpurun_out/summary_${W}_${TAG} > /dev/null
find $OUT -name "*.csv"
