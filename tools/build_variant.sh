#!/bin/bash
# A copy of the m2s package built from the CURRENT tree under variants/<name>/m2s (no stamps), for same-box
# A/B timing against the in-tree build (tools/ab_front.py).  Never used by tests, smoke or bench.
# Usage (repo root, CPU): bash tools/build_variant.sh <name>
set -e
ROOT=$(pwd)
NAME=${1:?variant name}
rm -rf variants/$NAME && mkdir -p variants/$NAME/m2s
cp mri-to-speech_amd/m2s/*.py variants/$NAME/m2s/
make -C mri-to-speech_amd/csrc -j8 OUT=$ROOT/variants/$NAME/m2s/libm2s.so TOUT=$ROOT/variants/$NAME/m2s/libm2s_torch.so \
  BUILD=build_variant_$NAME TLIBDIR=$ROOT/variants/$NAME/m2s
