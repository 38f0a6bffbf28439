"""render.hip's div_by -- IEEE x / d for 30 bands over one denominator via Markstein's correction
from RN(1 / d) -- must equal x / d bit for bit in its guarded range (tools/check_div.c, the same
float operations on the host: RN(1/d), a multiply, two FMAs)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_markstein_division_is_ieee(tmp_path):
    exe = str(tmp_path / "check_div")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(ROOT, "tools", "check_div.c"), "-lm"],
                   check=True)
    r = subprocess.run([exe, "20000000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert "differing 0" in r.stdout
