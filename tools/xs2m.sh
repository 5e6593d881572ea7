# A/B timing of experimental builds on the scan-to-map bench: tools/bench_s2m.py per library
#   bash tools/xs2m.sh lib1.so lib2.so ...   (paths relative to lego-loam-bor_amd/lego_amd)
mkdir -p gpurun_out/xs
for l in "$@"; do
  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$l timeout -k 10 300 python3 -u tools/bench_s2m.py --streams 256 --reps 5 --cpu-sample 1 > gpurun_out/xs/$l.log 2>&1 || exit 1
done
