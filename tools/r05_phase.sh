# Phase timers (profile build, -DLG_PROFILE) on the current code: C3 both VoxelGrid orders, C4 order 0.
#   python lego-loam-bor_amd/build.py --profile;  tools/r05_phase.sh TAG
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so
for O in 0 1; do
  timeout -k 10 300 python3 tools/phase_profile.py 256 $O > "$OUT/phase_order$O.txt" 2>&1
  grep "lm:\|voxel\|sort:\|LM solves\|heap" "$OUT/phase_order$O.txt"
done
timeout -k 10 300 python3 tools/phase_profile.py 256 0 hdl64 > "$OUT/phase_hdl64_order0.txt" 2>&1
grep "lm:\|voxel total\|LM solves" "$OUT/phase_hdl64_order0.txt"
echo done
