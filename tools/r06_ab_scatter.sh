set -e
OUT=gpurun_out/${TAG:-r06sc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for K in vlp16 hdl64; do
for L in ${VARS:-base noatom noscat}; do
  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_$L.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${K}_$L -o run -- python3 tools/proj_time.py $K 256 1 > $OUT/${K}_$L.log 2>&1
  grep proj_ms $OUT/${K}_$L.log
  f=$(find $OUT/${K}_$L -name '*kernel_stats.csv' | head -1); grep -E "k_pw_scatter|k_pw_columns|k_fa_prep4" $f | cut -d, -f1-4
done
done
