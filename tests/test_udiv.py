"""rc_udiv.h (the stream bodies' exact u64 division, rc_resume.hip) against the CPU's division:
edge values around every power of two and ~10^7 seeded pairs, built for the host with g++."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_udiv_matches_cpu_division(tmp_path):
    exe = tmp_path / "udiv_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "udiv_check.cpp")], check=True)
    out = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert int(out.stdout.strip()) > 10_000_000
