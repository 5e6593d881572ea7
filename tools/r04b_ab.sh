# Round-4 A/B of bench variants: each line "NAME|ENV|ARGS" runs bench.py once (no alt order).
#   tools/r04b_ab.sh TAG < variants.txt   (variants file in the repo: tools/ab/<name>.txt)
set -e
TAG=$1; VARS=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
while IFS='|' read -r NAME ENVS ARGS; do
  [ -z "$NAME" ] && continue
  env $ENVS timeout -k 10 200 python3 bench.py --no-cpu-baseline --roofline-streams 0 --no-alt-order $ARGS > "$OUT/$NAME.log" 2>&1
  tail -n 1 "$OUT/$NAME.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-24s %9.1f %6.3f' % ('$NAME', d['value'], d['ms_per_step']))"
done < "$VARS"
echo done
