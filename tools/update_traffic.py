"""Record the PMC-measured HBM traffic of a tools/profile.sh run for bench.py.

usage: python tools/update_traffic.py gpurun_out/prof_<tag> profiles/<tag>
Copies the kernel stats + counter summary into profiles/<tag>/ and stores
{workload: {fetch_bytes_x2, write_bytes, avg_ns, source}} in
profiles/pmc_traffic.json (bench.py's roofline.traffic; FETCH_SIZE doubled per
the gfx950 note in MI355X_MICROARCH.md, WRITE_SIZE as is, both per launch).
"""
import json
import shutil
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import summarize_prof  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]


def main(prof_dir, dest):
    prof_dir, dest = Path(prof_dir).resolve(), Path(dest).resolve()
    dest.mkdir(parents=True, exist_ok=True)
    bench_line = json.loads((prof_dir / "trace_bench.json").read_text().strip().splitlines()[-1])
    # the launch's dominant kernel: the brute-force sweep kernel, or the path kernel
    kname = bench_line["roofline"].get("kernel", "")
    kernel = "rt_brute_wf_kernel" if "rt_brute_wf_kernel" in kname else (
        "rt_brute_kernel" if "rt_brute_kernel" in kname else "rt_pathtrace_kernel")
    summ = summarize_prof.main(prof_dir, kernel)
    # bench.py prices a batch (rt_compute_frames' launch); the brute-force wavefront runs one
    # dispatch per (frame, bounce level) of the batch: its per-dispatch counters times that
    per_batch = 1
    if kernel == "rt_brute_wf_kernel":
        per_batch = int(bench_line["config"]["frame_batch"]) * max(1, int(bench_line["config"]["bounces"]))
        for k in ("fetch_bytes_x2", "write_bytes", "avg_ns"):
            if summ.get(k) is not None:
                summ[k] = summ[k] * per_batch
        summ["dispatches_per_batch"] = per_batch
    (dest / "summary.json").write_text(json.dumps(summ, indent=1) + "\n")
    ks = prof_dir / "trace" / "run_kernel_stats.csv"
    if ks.exists():
        shutil.copy(ks, dest / "kernel_stats.csv")
    shutil.copy(prof_dir / "trace_bench.json", dest / "trace_bench.json")
    key = f'{bench_line["config"]["workload"]} | frame_batch {bench_line["config"]["frame_batch"]}'
    f = ROOT / "profiles" / "pmc_traffic.json"
    table = json.loads(f.read_text()) if f.exists() else {}
    table[key] = {"fetch_bytes_x2": summ["fetch_bytes_x2"], "write_bytes": summ["write_bytes"],
                  "avg_ns": summ.get("avg_ns"), "valu_issue_util": summ.get("valu_issue_util"),
                  "valu_lane_util": summ.get("valu_lane_util"), "source": str(dest.relative_to(ROOT)),
                  "build_hash": bench_line["roofline"]["build_hash"]}  # the kernel build the counters came from
    f.write_text(json.dumps(table, indent=1, sort_keys=True) + "\n")
    print(json.dumps(table[key]))


if __name__ == "__main__":
    main(*sys.argv[1:])
