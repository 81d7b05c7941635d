"""bench.py's printed line: it must reach the driver whole (the driver keeps the last 8000 bytes
of stdout), carry the headline, roofline, cpu_baseline and every leg, and label the dominant
kernel with the arithmetic it really runs."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _row(i):
    return {"cls": f"convT 128->128 k3 s1 [4x16x16x16] variant {i:03d}", "kernels": "conv_brick_x3(op16);wgrad_reduce",
            "launches_per_step": 36, "ms_per_step": 1.0 / (i + 1), "mean_us": 32.8, "frac": 0.175}


def _leg(n_rows):
    return {"value": 30.0, "unit": "patches/s", "ms_per_step": 33.0, "ms_per_step_median": 32.9, "dtype": "bf16",
            "dtype_detail": "x" * 200, "workload": "y" * 120, "step_launch": "hip_graph",
            "step_roofline": {"achieved": 0.2, "ideal_ms": 8.0, "formula": "z" * 60, "note": "n" * 120, "F_tflop": 12.9,
                              "P_mfma_tflops": 2516.6, "B_ew_gb": 23.7, "B_ew_elem_bytes": 2, "BW_hbm_gbs": 8000.0,
                              "achieved_fp32_storage": 0.33},
            "roofline": {"bound": "mfma", "kernel": "conv_brick_x3(op16) (bf16 MFMA) - convT", "achieved": 450.0,
                         "peak": 2516.6, "unit": "TFLOP/s", "frac": 0.18, "traffic": None, "timing": "t" * 150,
                         "launch_ms": 0.12, "launches_per_step": 36},
            "alt_precisions": {"bf16x3": {"value": 17.1, "ms_per_step": 58.3, "ms_per_step_median": 58.3,
                                          "dtype": "bf16x3"}},
            "top_kernels": [_row(i) for i in range(n_rows)], "kernel_ms_per_step_serial": 38.0,
            "config": {"patch": 128, "batch": 1, "nc": 1, "netG": "resnet_9blocks", "conv_precision": "bf16"}}


def test_line_fits_driver_tail(tmp_path):
    b = _bench()
    head = _leg(200)
    res = {"metric": "3D patches/sec per CycleGAN step (G+D fwd+bwd)", "value": 172.4, "unit": "patches/s",
           "roofline": head["roofline"], "step_roofline": head["step_roofline"], "top_kernels": head["top_kernels"],
           "legs": {f"leg{i}": _leg(60) for i in range(4)},
           "cpu_baseline": {"value": 0.58, "unit": "patches/s", "cores": 16, "kind": "port", "sample": "s" * 250}}
    full = tmp_path / "full.json"
    out = b.compact_line(res, str(full))
    line = json.dumps(out)
    assert len(line) <= b.LINE_CAP < 8000
    back = json.loads(line)
    for k in ("value", "roofline", "cpu_baseline", "legs"):
        assert k in back
    assert set(back["legs"]) == set(res["legs"])
    assert all("roofline" in leg and "value" in leg for leg in back["legs"].values())
    assert len(back["top_kernels"]) >= 3
    # the whole report is on disk, every row of every leg
    stored = json.loads(full.read_text())
    assert len(stored["top_kernels"]) == 200
    assert all(len(leg["top_kernels"]) == 60 for leg in stored["legs"].values())


def test_kernel_arith_labels():
    b = _bench()
    assert b.kernel_arith("thin_n_tile8", "bf16").startswith("VALU dot")
    assert "fp64" in b.kernel_arith("thin_n_tile8", "bf16")
    assert b.kernel_arith("thin_dot", "fp16") == "VALU dot, fp16-rounded operands, f32 accumulate"
    assert b.kernel_arith("brickT_pack;brickT_x3(op16)", "bf16") == "bf16 MFMA"
    assert b.kernel_arith("conv_brick_x3(op16)", "bf16x3") == "bf16x3 split MFMA"
    assert b.kernel_arith("in_bwd_stats;in_bwd_finalize;in_bwd_apply(op16)", "bf16") == "HBM-bound elementwise"
