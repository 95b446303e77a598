mkdir -p gpurun_out/x1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "effnet or pipeline or smoke" > gpurun_out/x1/pytest.log 2>&1 && \
for m in 0 1 4 8; do timeout -k 10 60 ./tools/halo_bench_$m || exit 1; done > gpurun_out/x1/halo.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/x1/bench.json 2> gpurun_out/x1/bench.err
rc=$?; tail -2 gpurun_out/x1/pytest.log; cat gpurun_out/x1/halo.log; cat gpurun_out/x1/bench.json; exit $rc
