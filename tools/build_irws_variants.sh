#!/bin/bash
# ir_ws scheduling variants for a same-box A/B (tools/ab_kern.py): each is the in-tree build with ir_ws.hip
# recompiled under other IRWS_* switches, under variants/<name>/m2s.  Diagnostic only.  Usage (repo root, CPU):
#   bash tools/build_irws_variants.sh name:"-DIRWS_HAND_END=0 -DIRWS_TAPS_AHEAD=0" ...
set -e
ROOT=$(pwd)
for spec in "$@"; do
  NAME=${spec%%:*}; FL=${spec#*:}
  B=mri-to-speech_amd/csrc/build_variant_$NAME
  rm -rf variants/$NAME $B && mkdir -p variants/$NAME/m2s $B
  cp mri-to-speech_amd/m2s/*.py variants/$NAME/m2s/
  for o in mri-to-speech_amd/csrc/build/*.o; do [ "$(basename $o)" = "${SRC:-ir_ws.hip}.o" ] || cp -p $o $B/; done
  make -s -C mri-to-speech_amd/csrc -j8 OUT=$ROOT/variants/$NAME/m2s/libm2s.so TOUT=$ROOT/variants/$NAME/m2s/libm2s_torch.so \
    BUILD=build_variant_$NAME TLIBDIR=$ROOT/variants/$NAME/m2s EXTRA="$FL"
done
