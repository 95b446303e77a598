#!/bin/bash
# Per-file compile-flag variants for a same-box A/B (tools/ab_kern.py / ab_pipe_kern.py): each variant is the in-tree build
# with ONE source recompiled under other flags (NOSLP overrides the Makefile's -fno-slp-vectorize list).  Diagnostic only.
# Usage (repo root, CPU):  bash tools/build_flag_variants.sh name:src.hip:"extra flags":"noslp list" ...
set -e
ROOT=$(pwd)
for spec in "$@"; do
  IFS=: read -r NAME SRCF FL NS <<< "$spec"
  B=mri-to-speech_amd/csrc/build_variant_$NAME
  rm -rf variants/$NAME $B && mkdir -p variants/$NAME/m2s $B
  cp mri-to-speech_amd/m2s/*.py variants/$NAME/m2s/
  for o in mri-to-speech_amd/csrc/build/*.o; do [ "$(basename $o)" = "$SRCF.o" ] || cp -p $o $B/; done
  make -s -C mri-to-speech_amd/csrc -j8 OUT=$ROOT/variants/$NAME/m2s/libm2s.so TOUT=$ROOT/variants/$NAME/m2s/libm2s_torch.so \
    BUILD=build_variant_$NAME TLIBDIR=$ROOT/variants/$NAME/m2s EXTRA="$FL" NOSLP="$NS"
done
