#!/bin/bash
set -o pipefail
TAG=${1:-r06l}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "bilstm" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 200 python -u tools/lstm_bench.py bf16x3 > "$OUT/lstm_x3g.txt" 2>&1 || { tail -20 "$OUT/lstm_x3g.txt"; exit 1; }
M2S_LSTM_X3G=0 timeout -k 10 200 python -u tools/lstm_bench.py bf16x3 > "$OUT/lstm_x3.txt" 2>&1 || { tail -20 "$OUT/lstm_x3.txt"; exit 1; }
grep bilstm "$OUT/lstm_x3g.txt"; grep bilstm "$OUT/lstm_x3.txt"
