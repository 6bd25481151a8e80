"""utils/plots.py: the data shaping behind the harness chart and the scaling
figure (pure pandas / lists), and that both figures are written."""
import pandas as pd

from cuda_mpi_openmp_amd.utils import plots


def _runs():
    rows = []
    for ks, ms in (([[1, 32], [1, 32]], [2.0, 4.0, 3.0]), ([[64, 64], [32, 32]], [1.0, 1.0])):
        rows += [{"device": "HIP", "kernel_size": ks, "time_kernel_exe_ms": t, "filename": "a.data"} for t in ms]
    rows += [{"device": "CPU", "kernel_size": [None, None], "time_kernel_exe_ms": t, "filename": "a.data"}
             for t in (10.0, 30.0)]
    return pd.DataFrame(rows)


def test_median_groups_order_and_labels():
    g = plots.median_groups(_runs())
    assert list(g["label"]) == ["HIP_[[1, 32], [1, 32]]", "HIP_[[64, 64], [32, 32]]", "CPU"]
    assert list(g["median_ms"]) == [3.0, 1.0, 20.0]
    assert list(g["samples"]) == [3, 2, 2]
    note = plots.metadata_note(_runs(), ["filename", "absent"], g)
    assert "filename: [a.data]" in note and "CPU: 2 samples" in note and "absent" not in note


def test_scaling_series():
    rows = [{"name": "conv", "kind": "weak", "n": n, "status": "ok", "value": v} for n, v in ((1, 10.0), (2, 19.0))]
    rows += [{"name": "jacobi", "kind": "strong", "n": n, "status": "ok", "speedup": s} for n, s in ((1, 1.0), (2, 1.8))]
    rows += [{"name": "skip", "kind": "weak", "n": 2, "status": "skipped"}]
    weak, strong = plots.scaling_series(rows)
    assert weak == {"conv": [(1, 1.0), (2, 1.9)]} and strong == {"jacobi": [(1, 1.0), (2, 1.8)]}


def test_figures_written(tmp_path):
    g = plots.median_groups(_runs())
    a = plots.annotated_bars(g["label"], g["median_ms"], str(tmp_path / "m.png"), note="x", title="t")
    rows = [{"name": "conv", "kind": "weak", "n": n, "status": "ok", "value": v} for n, v in ((1, 10.0), (2, 19.0))]
    b = plots.scaling_figure(rows, str(tmp_path / "s.png"), "t")
    for p in (a, b):
        assert p is None or (tmp_path / p.split("/")[-1]).stat().st_size > 1000
