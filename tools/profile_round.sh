#!/bin/bash
# Profile bench.py's hot path (run on the GPU box from the repo root):
#   rocprofv3 --kernel-trace --stats, then FETCH_SIZE and WRITE_SIZE in their
#   own --pmc passes (MI355X_MICROARCH.md §HBM).  Only gpurun_out/ comes back
#   from the box: run tools/pmc_summary.py here afterwards to write profiles/.
# usage: bash tools/profile_round.sh <round> <config> [content: band4 | noise | static]
set -e
R=${1:-r02}; C=${2:-4k}; K=${3:-band4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SFX=$( [ "$K" = band4 ] || echo _$K )
OUT=gpurun_out/prof_$C$SFX
rm -rf $OUT && mkdir -p $OUT
# bench.py's default steps / warm-up; no per-frame check (it adds host work, not GPU work)
ARGS="--config $C --content $K --no-verify --no-end-to-end --no-cpu-baseline --no-api --no-host-rgb"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_kt -o run -- python3 bench.py $ARGS > $OUT/prof_kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_fetch -o run -- python3 bench.py $ARGS > $OUT/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_write -o run -- python3 bench.py $ARGS > $OUT/prof_write.log 2>&1
# wave states of the engine (8 SQ counters + GRBM_GUI_ACTIVE, one pass)
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/prof_sq -o run -- python3 bench.py $ARGS > $OUT/prof_sq.log 2>&1
# LDS: instructions, bank-conflict and unaligned-stall cycles against all
# LDS-array cycles, and the waves' LDS issue stalls
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/prof_lds -o run -- python3 bench.py $ARGS > $OUT/prof_lds.log 2>&1
# read requests by size, and the uncached 32-byte ones (the hand-off polls and
# granule loads), so the traffic needs no blanket FETCH_SIZE correction
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RD_UNCACHED_32B_sum --output-format csv -d $OUT/prof_rdsize -o run -- python3 bench.py $ARGS > $OUT/prof_rdsize.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/prof_req -o run -- python3 bench.py $ARGS > $OUT/prof_req.log 2>&1
# L2 (TCC) hits and misses of the reads and writes the CUs send it: the hit
# rate says how much of the requested window / poll traffic the XCD L2s absorb
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_WRITE_sum --output-format csv -d $OUT/prof_hit -o run -- python3 bench.py $ARGS > $OUT/prof_hit.log 2>&1
echo "profiled $R $C $K: now run python tools/pmc_summary.py --round $R --config $C --content $K --src $OUT locally"
