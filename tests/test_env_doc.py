"""docs/ENV.md lists every REPLICANN_* environment variable the sources read (and no stale ones)."""

import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _knobs_in_sources():
    found = set()
    for pat in ("csrc/**/*.hip", "csrc/**/*.h", "csrc/**/*.cpp", "replicann_amd/**/*.py", "bench.py"):
        for f in ROOT.glob(pat):
            found |= set(re.findall(r"REPLICANN_[A-Z0-9_]*[A-Z0-9]", f.read_text(errors="ignore")))
    return found


def test_every_knob_documented():
    doc = (ROOT / "docs" / "ENV.md").read_text()
    documented = set(re.findall(r"REPLICANN_[A-Z0-9_]*[A-Z0-9]", doc))
    used = _knobs_in_sources()
    assert used, "no knobs found: source globs broken"
    assert not used - documented, f"undocumented: {sorted(used - documented)}"
    assert not documented - used, f"documented but never read: {sorted(documented - used)}"
