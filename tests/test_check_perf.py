"""T6: the perf-regression comparison logic (scripts/check_perf.py) on synthetic bench lines."""

import importlib.util
import io
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _mod():
    spec = importlib.util.spec_from_file_location("check_perf", ROOT / "scripts" / "check_perf.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _line(model, value, n=1):
    return {"metric": "x", "value": value, "unit": "samples/s", "n_gpus": n, "config": {"model": model}}


def test_check_perf_pass_fail_skip(monkeypatch, capsys):
    m = _mod()
    base = json.loads((ROOT / "scripts" / "perf_baseline_r2.json").read_text())
    want = base["gpt2-small"]["value"]
    assert m.check(_line("gpt2-small", want * 0.97), base, 0.05)[0]
    assert not m.check(_line("gpt2-small", want * 0.90), base, 0.05)[0]
    assert m.check(_line("gpt2-small", 1.0, n=8), base, 0.05)[0]  # multi-GPU lines are not compared
    assert m.check(_line("no-such-model", 1.0), base, 0.05)[0]
    monkeypatch.setattr(sys, "stdin", io.StringIO(json.dumps(_line("gpt2-small", want * 0.5)) + "\n"))
    assert m.main([]) == 1
    assert "FAIL gpt2-small" in capsys.readouterr().out
