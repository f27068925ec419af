"""Copy the judged evidence of tools/refresh_profiles.sh (gpurun_out/refresh)
into profiles/<round>/ and regenerate profiles/pmc_*.json (roofline.traffic).
usage: python tools/collect_profiles.py r01"""
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "gpurun_out", "refresh")
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
dst = os.path.join(ROOT, "profiles", tag)
os.makedirs(dst, exist_ok=True)
for f in ["pytest_gpu.log", "smoke.log", "bench_b4096_f64.json", "bench_b65536_f32.json"]:
    shutil.copy(os.path.join(src, f), os.path.join(dst, f))
for d, name in [("prof_f64", "kernel_stats_b4096_f64.csv"), ("prof_f32", "kernel_stats_b65536_f32.csv")]:
    hits = glob.glob(os.path.join(src, d, "**", "*kernel_stats.csv"), recursive=True)
    if hits:
        shutil.copy(hits[0], os.path.join(dst, name))
hits = glob.glob(os.path.join(src, "prof_col_c2", "**", "*kernel_stats.csv"), recursive=True)
if hits:
    os.makedirs(os.path.join(dst, "collision"), exist_ok=True)
    shutil.copy(hits[0], os.path.join(dst, "collision", "kernel_stats_c2_f64.csv"))
for sub in ["collision", "matrix"]:
    os.makedirs(os.path.join(dst, sub), exist_ok=True)
    for f in glob.glob(os.path.join(src, sub, "*.json")):
        shutil.copy(f, os.path.join(dst, sub, os.path.basename(f)))
for B, dt in [(4096, "f64"), (65536, "f32")]:
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), os.path.join(src, "pmc"), dt,
                    str(B), tag], check=True)
print("collected into", dst)
