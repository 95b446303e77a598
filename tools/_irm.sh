#!/bin/bash
# ir_pwdw MFMA-depthwise check: fused-IR parity tests, microbench (0 = library, 128 = VALU depthwise), bench
OUT=gpurun_out/irm; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ir_fused or fused_kernels or pipeline or effnet_bf16" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& for m in 0 128; do timeout -k 10 60 ./tools/irf_bench_$m || exit 1; done > $OUT/ab.log 2>&1 \
&& timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; tail -3 $OUT/pytest.log; cat $OUT/ab.log; cat $OUT/bench.json; exit $rc
