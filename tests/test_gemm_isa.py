"""ISA-level guard for the persistent GEMM's dynamic tile queue (csrc/include/gemm_pk.h).

Wave 0's schedule atomic returns its value into a VGPR asynchronously, invisible to hipcc's
waitcnt insertion; the value is read only after the counted wait that retires it.  That is sound
only if the compiler neither copies nor reuses that register between the issue and the read — a
property of register allocation, so it is checked here on the generated code of every
instantiation (a violation once produced garbage tile ids and a hung GEMM).  CPU-only: hipcc
cross-compiles gfx950."""

import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
TUS = ["gemm_pk_tt_dyn", "gemm_pk_tf_dyn", "gemm_pk_ff_dyn", "gemm_pk_ft_dyn"]


@pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not available")
def test_schedule_register_never_touched_in_flight(tmp_path):
    def comp(tu):
        out = tmp_path / f"{tu}.s"
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast",
                            "-munsafe-fp-atomics", f"-I{ROOT / 'csrc' / 'include'}", "-S", "--offload-device-only",
                            str(ROOT / "csrc" / "kernels" / f"{tu}.hip"), "-o", str(out)],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]
        return out
    with ThreadPoolExecutor(len(TUS)) as ex:
        outs = list(ex.map(comp, TUS))
    r = subprocess.run([sys.executable, str(ROOT / "tests" / "tools" / "gemm_deq_check.py"), *map(str, outs)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-4000:]
    assert r.stdout.count(" OK") >= 20  # every dynamic instantiation was checked and passed
