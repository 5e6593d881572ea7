# Schedule / sort A/B on the GPU: the quick parity suite, then bench lines for environment variants.
#   tools/r04_ab.sh TAG "pytest -k expression" "VAR=1 VAR2=0" "VAR=1" ...   ("-" = no variables)
set -e
TAG=$1; KEXPR=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$KEXPR" > "$OUT/tests.log" 2>&1
  tail -3 "$OUT/tests.log"
fi
i=0
for v in "$@"; do
  i=$((i+1))
  if [ "$v" = "-" ]; then v=""; fi
  env $v timeout -k 10 300 python3 bench.py --no-cpu-baseline --roofline-streams 0 > "$OUT/bench$i.log" 2>&1
  echo "[$i] $v: $(grep -o '"value": [0-9.]*' "$OUT/bench$i.log" | head -1) alt $(grep -o '"other_voxel_tie_order": {[^}]*}' "$OUT/bench$i.log")"
done
echo done
