#!/bin/bash
# Round 6: lstm_x3g (granule hand-off, 5..16 sequences) tests and timing; the ir_ws per-parity variant A/B.
set -o pipefail
TAG=${1:-r06k}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs4.py tests/test_gpu_bf16x3.py -m gpu -x -q \
  -k "bilstm or timeout or config4 or ir_ws" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 200 python -u tools/lstm_bench.py bf16x3 > "$OUT/lstm_x3g.txt" 2>&1 || { tail -20 "$OUT/lstm_x3g.txt"; exit 1; }
M2S_LSTM_X3G=0 timeout -k 10 200 python -u tools/lstm_bench.py bf16x3 > "$OUT/lstm_x3.txt" 2>&1 || { tail -20 "$OUT/lstm_x3.txt"; exit 1; }
grep bilstm "$OUT/lstm_x3g.txt"; grep bilstm "$OUT/lstm_x3.txt"
AB_ROUNDS=3 timeout -k 10 400 python -u tools/ab_kern.py mri-to-speech_amd variants/par1 > "$OUT/ab_par.txt" 2>&1 || { tail -20 "$OUT/ab_par.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_par.txt"
