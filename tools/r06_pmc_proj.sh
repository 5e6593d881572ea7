# Round 6: SQ / memory counters of the projection-only timing (tools/proj_time.py), one pass each.
#   tools/r06_pmc_proj.sh TAG KIND [LIB]
set -e
OUT=gpurun_out/$1; K=$2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ -n "$3" ] && export LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $OUT/sq_$K -o run -- python3 tools/proj_time.py $K 256 1 > $OUT/sq_$K.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$K -o run -- python3 tools/proj_time.py $K 256 1 > $OUT/fetch_$K.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_$K -o run -- python3 tools/proj_time.py $K 256 1 > $OUT/write_$K.log 2>&1
python3 tools/pmc_agg.py $OUT/sq_$K $OUT/fetch_$K $OUT/write_$K
