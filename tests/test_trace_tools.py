"""tools/step_timeline.py and tools/queue_report.py on a synthetic rocprofv3 kernel trace (CSV and
the rocpd SQLite layout): per-queue busy time, overlap, GPU-idle holes and the kernel classes."""
import csv
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# two steps; main chain on queue 1, weight gradients on queue 4, one comm kernel on queue 4
KERNELS = []
for step in range(3):
    t = step * 1000_000
    KERNELS += [(t, t + 100_000, 1, "dbx::augment_u8_kernel(...)"),
                (t + 100_000, t + 500_000, 1, "void dbx::igemm_kernel<128, 128>(dbx::IGemmArgs)"),
                (t + 200_000, t + 600_000, 4, "void dbx::wgrad_dma_kernel<256, 256>(dbx::WgradArgs)"),
                (t + 600_000, t + 650_000, 4, "ncclDevKernel_AllReduce(...)"),
                (t + 700_000, t + 900_000, 1, "dbx::sgd_kernel(...)")]


def _csv(tmp_path):
    p = tmp_path / "run_kernel_trace.csv"
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Start_Timestamp", "End_Timestamp", "Queue_Id", "Kernel_Name"])
        for r in KERNELS:
            w.writerow(r)
    return str(p)


def _db(tmp_path):
    p = tmp_path / "run_results.db"
    with sqlite3.connect(p) as c:
        c.execute("create table kernels (start integer, end integer, queue_id integer, name text)")
        c.executemany("insert into kernels values (?, ?, ?, ?)", KERNELS)
    return str(p)


def _run(tool, *args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", tool), *args], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_step_timeline_csv_and_db(tmp_path):
    for src in (_csv(tmp_path), _db(tmp_path)):
        out = _run("step_timeline.py", src, "--steps", "1", "--tail", "2", "--gap-us", "50")
        assert "wall 1.000 ms" in out and "queue 1: busy 0.700 ms" in out and "queue 4: busy 0.450 ms" in out
        assert "both queues busy 0.300 ms" in out
        assert "GPU idle (no queue busy): 0.150 ms" in out  # 650-700 us and 900-1000 us


def test_queue_report_classes(tmp_path):
    out = _run("queue_report.py", _db(tmp_path), "--steps", "2")
    assert "queue 1: main 6" in out and "queue 4: wgrad 2, comm 2" in out
    assert "shared: [4]" in out
