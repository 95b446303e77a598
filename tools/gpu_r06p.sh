#!/bin/bash
# Round 6: small-pass changes (stem strip parts, SE excitation fold): parity tests (KSEL) and the small-shape timings
# against the settings in ABSET.
set -o pipefail
TAG=${1:-r06p}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${KSEL:-stem or config2 or config1 or effnet_bf16x3_every_block or se_excitation}" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/ab_small.py "" ${ABSET:-"M2S_STEM_PARTS=1"} > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v "^#" "$OUT/ab.txt"
if [ -n "$TIMELINE" ]; then bash tools/gpu_small.sh "$TAG/small" || exit 1; fi
if [ -n "$BENCH" ]; then bash tools/ab_bench_stages.sh "$TAG/bench" M2S_DUMMY_SWITCH 1 "0" || exit 1; fi
if [ -n "$GRAPH" ]; then timeout -k 10 300 python -u tools/graph_small.py > "$OUT/graph.txt" 2>&1 || { tail -20 "$OUT/graph.txt"; exit 1; }; grep -v "^#" "$OUT/graph.txt"; fi
