"""bin/pipeline at C3 size: 500,149 bp genome (1M windows), 100k reads as FASTQ,
index built by bin/hnswpq_index. Prints the CLI's stage times next to the kernel time of the same work
(the executor's device span). Run on the GPU box: python tools/scripts/pipeline_c3.py [workdir] [extra env]"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from deepreadmapper_amd import synth  # noqa: E402

wd = sys.argv[1] if len(sys.argv) > 1 else "/tmp/drm_pipeline_c3"
os.makedirs(wd, exist_ok=True)
g = synth.genome(500_149, seed=42)
fna, fq = os.path.join(wd, "c3.fna"), os.path.join(wd, "c3.fastq")
if not os.path.exists(fq):
    synth.write_fasta(fna, g)
    reads, names, _ = synth.simulate_reads(g, 100_000, seed=7)
    synth.write_fastq(fq, reads, names)
if not os.path.exists(os.path.join(wd, "c3idx", "config.txt")):
    t0 = time.time()
    subprocess.run([os.path.join(ROOT, "bin", "hnswpq_index"), fna, "c3idx", "150"], cwd=wd, check=True,
                   stdout=subprocess.DEVNULL)
    print(f"hnswpq_index: {time.time() - t0:.1f} s", flush=True)
for rep in range(2):
    t0 = time.time()
    r = subprocess.run([os.path.join(ROOT, "bin", "pipeline"), "c3idx", fq, fna, "128", "128", "5", "out"], cwd=wd,
                       capture_output=True, text=True)
    if r.returncode != 0:
        print(r.stdout, r.stderr)
        sys.exit(1)
    print(f"run {rep}: wall {time.time() - t0:.1f} s")
    print("\n".join(l for l in r.stdout.split("\n") if "time" in l.lower()), flush=True)
    print("\n".join(l for l in r.stderr.split("\n") if l.startswith("[exec]")), flush=True)
