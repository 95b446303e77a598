#!/bin/bash
# Round 6: rb1_fused row-wide epilogue stores: vocoder parity tests, same-box A/B against the per-lane 8-byte stores
# (variants/rowst0: -DRB1_ROWST=0), and the LDS conflict counters of the bf16x3 step's rb1 launches.
set -o pipefail
TAG=${1:-r06n}
ROOT=$(pwd)
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "vocoder or mrf" \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
AB_DTYPES=bf16x3,fp8 timeout -k 10 600 python -u tools/ab_pipe_kern.py mri-to-speech_amd variants/rowst0 > "$OUT/ab.txt" 2>&1 \
  || { cat "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt"
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE --output-format csv \
  -d "$ROOT/$OUT/pmc" -o run -- python3 "$ROOT/tools/ab_step.py" --child mri-to-speech_amd bf16x3) > "$OUT/pmc.log" 2>&1 \
  || { tail -20 "$OUT/pmc.log"; exit 1; }
python3 - "$OUT/pmc" <<'PY'
import csv, glob, os, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection*.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "rb1" in k or "conv1d_halo" in k:
            acc[k.split("(")[0][-60:]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(acc.items()):
    print(f"{k:60s} conflicts/lds_inst {v['SQ_LDS_BANK_CONFLICT'] / max(v['SQ_INSTS_LDS'], 1):.3f}  conflicts/idx_active {v['SQ_LDS_BANK_CONFLICT'] / max(v['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
PY
