"""tools/evidence.py's stage alignment (CPU): the rocprofv3 dispatches of a PMC pass are matched, in order, with the
stage-tagged launch log libm2s kept for the profiled steps, past the set-up dispatches the trace also holds."""
import csv
import importlib.util
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _evidence():
    spec = importlib.util.spec_from_file_location("evidence", os.path.join(REPO, "tools", "evidence.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _pass(tmp_path, dispatches, launches, steps=2):
    d = tmp_path / "fetch"
    d.mkdir()
    with open(d / "run_counter_collection.csv", "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for i, (name, v) in enumerate(dispatches, start=1):
            w.writerow([i, name, "FETCH_SIZE", v])
    with open(str(d) + ".launches.json", "w") as fh:
        json.dump({"steps": steps, "launches": launches}, fh)
    return str(d)


def test_stage_alignment_skips_setup_dispatches(tmp_path):
    ev = _evidence()
    setup = [("pack_kernel(float const*)", 1.0)] * 20 + [("stem_b0_kernel<16, 1>(m2s::StemB0Args)", 5.0)]  # a set-up use
    step = [("stem_b0_kernel<16, 1>(m2s::StemB0Args)", 10.0), ("__amd_rocclr_fillBufferAligned", 0.5),
            ("ir_ws_kernel<16, 4, 1>(bf16 const*)", 20.0), ("conv_gemm_kernel<128, 128>(args)", 3.0)]
    launches = [["stem_b0_kernel<16, 1>", "cnn"], ["ir_ws_kernel<16, 4, 1>", "cnn"], ["conv_gemm_kernel<128, 128>", "mrf_c256"]]
    d = _pass(tmp_path, setup + step + step, launches * 2)
    st_map, steps, matched, n = ev.dispatch_stages(d)
    assert steps == 2 and matched == n == 6
    agg = ev.stage_counters(d, st_map)
    assert agg["cnn"]["FETCH_SIZE"] == 60.0 and agg["mrf_c256"]["FETCH_SIZE"] == 6.0  # no set-up dispatch counted
