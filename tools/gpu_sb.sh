#!/bin/bash
# ir_s2band (banded stride-2 IR front half, blocks.3.0): parity tests, then kernel stats with it on / off for the
# bf16x3 bench step, and the fp8 engine at 8 x 1000 frames with it on.  Usage: bash tools/gpu_sb.sh <tag>
set -o pipefail
TAG=${1:-sb}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread \
  -k "s2band or bf16x3_every_block or pipeline_bf16x3 or fp8 or ir_fused or bf16_close or config" > "$OUT/pytest.log" 2>&1 \
  || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"; grep -E " cos " "$OUT/pytest.log" | cut -c1-150
bash tools/gpu_se_ab.sh "$TAG/x3" "M2S_IR_S2BAND=1" "M2S_IR_S2BAND=0" > /dev/null || exit 1
grep -E "total|ir_s2band|dwconv_kernel<m2s::sp_t, 2>|conv_gemm_kernel<128, 128, 4, 4, 2, 3, 0, 1>" "$OUT/x3/v1.txt" "$OUT/x3/v2.txt"
for sb in 1 0; do
  (cd /tmp && M2S_IR_S2BAND=$sb CLIPS=8 FRAMES=1000 CHUNK=1920 STEPS=2 DTYPE=fp8 timeout -k 10 180 rocprofv3 --kernel-trace --stats \
     --output-format csv -d "$ROOT/$OUT/fp8_$sb" -o run -- python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/fp8_$sb.log" 2>&1) || exit 1
  python3 tools/kstats.py "$OUT/fp8_$sb" 2 > "$OUT/fp8_$sb.txt"; echo "== fp8 s2band=$sb"
  grep -E "total|ir_s2band|dwconv_kernel<unsigned short, 2>|conv_gemm_kernel<128, 256, 4, 8, 2, 3, 0, 0>" "$OUT/fp8_$sb.txt"
done
