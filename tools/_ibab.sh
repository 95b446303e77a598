#!/bin/bash
# ir_block ablation: time ir_block_kernel for each prebuilt IB_MODE variant (m2s/libm2s_ib<v>.so)
OUT=gpurun_out/ibab
mkdir -p $OUT
export TMPDIR=/tmp
cp mri-to-speech_amd/m2s/libm2s.so /tmp/libm2s_keep.so
rc=0
for v in ${@:-0 1 2 4 8 16 31}; do
  cp mri-to-speech_amd/m2s/libm2s_ib$v.so mri-to-speech_amd/m2s/libm2s.so
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/$OUT/v$v -o run -- python3 /root/repo/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > /root/repo/$OUT/v$v.log 2>&1) || { rc=$?; break; }
  python3 tools/kstats.py $OUT/v$v 2 ${ABF:-ir_block} 2>/dev/null | sed -n 2,4p | sed "s/^/v$v /"
done
cp /tmp/libm2s_keep.so mri-to-speech_amd/m2s/libm2s.so
exit $rc
