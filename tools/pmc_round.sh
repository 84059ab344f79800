#!/bin/bash
# PMC passes for the round's profiles (GPU box): FETCH_SIZE / WRITE_SIZE (separate passes, gfx950
# corrections in tools/pmc_summary.py) and an L2 hit/miss pass per config, plus an SQ pass over the
# particle encoders.  Usage: tools/pmc_round.sh TAG   (writes gpurun_out/pmc_TAG_*)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
tag=$1
run() {   # name "counters" bench-args
  timeout -s KILL 150 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/pmc_${tag}_$1 -o run -- python3 bench.py $3 \
    > gpurun_out/pmc_${tag}_$1.log 2>&1 || { echo "pass $1 failed"; tail -5 gpurun_out/pmc_${tag}_$1.log; exit 1; }
  echo "pass $1 ok"
}
H="--config humanoid --steps 20 --warmup 5"
P="--config particles --steps 2 --warmup 1"
C="--steps 40 --warmup 10"
L="--config pendulum --steps 40 --warmup 10"
run hf FETCH_SIZE "$H" && run hw WRITE_SIZE "$H" && run hl "TCC_HIT_sum TCC_MISS_sum" "$H" && \
run pf FETCH_SIZE "$P" && run pw WRITE_SIZE "$P" && \
run ps "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" "$P" && \
run cf FETCH_SIZE "$C" && run cw WRITE_SIZE "$C" && \
run lf FETCH_SIZE "$L" && run lw WRITE_SIZE "$L"
