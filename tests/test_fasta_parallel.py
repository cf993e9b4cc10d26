"""The CLI's parallel FASTA ingest against the sequential reader (CPU)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parallel_fasta_ingest_equals_sequential_reader(tmp_path):
    exe = tmp_path / "fasta_fuzz"
    subprocess.run(["g++", "-O1", "-std=c++17", "-pthread", os.path.join(ROOT, "tests", "fasta_fuzz.cpp"), "-o",
                    str(exe)], check=True)
    p = subprocess.run([str(exe), str(tmp_path / "x.fa")], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and p.stdout.strip().endswith("OK"), p.stdout[-2000:]
