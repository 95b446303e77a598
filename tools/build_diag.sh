#!/bin/bash
# Diagnostic copy of the m2s package with in-kernel stamps compiled in (-DIRWS_TRACE), under diag/m2s/,
# so a diagnostic run imports it ahead of the real package (tools/trace_ir_ws.py puts diag/ first on
# sys.path).  Never used by tests, smoke or bench.  Usage: bash tools/build_diag.sh  (repo root, CPU)
set -e
ROOT=$(pwd)
rm -rf diag && mkdir -p diag/m2s
cp mri-to-speech_amd/m2s/*.py diag/m2s/
make -C mri-to-speech_amd/csrc -j8 OUT=$ROOT/diag/m2s/libm2s.so TOUT=$ROOT/diag/m2s/libm2s_torch.so \
  BUILD=build_diag EXTRA=-DIRWS_TRACE TLIBDIR=$ROOT/diag/m2s
