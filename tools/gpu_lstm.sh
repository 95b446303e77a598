#!/bin/bash
# BiLSTM split-kernel check on the GPU box: parity tests, then per-step timing of both B > 16 kernels.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-lstm}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "bilstm" > "$OUT/pytest.log" 2>&1 \
&& timeout -k 10 120 python -u tools/lstm_bench.py bf16x3 > "$OUT/x3.txt" 2>&1 \
&& M2S_LSTM_X3=0 timeout -k 10 120 python -u tools/lstm_bench.py bf16x3 > "$OUT/f32.txt" 2>&1
rc=$?
tail -5 "$OUT/pytest.log"; cat "$OUT/x3.txt" "$OUT/f32.txt" 2>/dev/null
exit $rc
