# r04_ab.sh plus a second parity pass with LEGO_LM_GRID=3 (the grid search for staged clouds too)
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LEGO_LM_GRID=3 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not test_gpu_long and not long_sequence" > "$OUT/tests_grid3.log" 2>&1
tail -3 "$OUT/tests_grid3.log"
bash tools/r04_ab.sh "$@"
