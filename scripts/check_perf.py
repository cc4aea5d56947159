"""T6 perf regression check: a bench.py JSON line against the committed floor.

    python bench.py --model gpt2-small | python scripts/check_perf.py            # from stdin
    python scripts/check_perf.py --run gpt2-small vit-b16 [--tolerance 0.05]       # runs bench.py itself

Per config: PASS if value >= baseline * (1 - tolerance) (default 5 %: MI355X boxes differ by up to
~3 % in sustained clock), else FAIL; exit status 1 if any config fails.  Baselines:
scripts/perf_baseline_r2.json.  Only single-GPU lines are compared (n_gpus == 1)."""

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASELINE = os.path.join(ROOT, "scripts", "perf_baseline_r2.json")


def check(line: dict, baseline: dict, tolerance: float):
    """(ok, message) for one bench JSON record."""
    model = line.get("config", {}).get("model")
    if model not in baseline:
        return True, f"SKIP {model}: no committed baseline"
    if line.get("n_gpus") != 1:
        return True, f"SKIP {model}: n_gpus={line.get('n_gpus')} (baselines are 1-GPU)"
    want = baseline[model]["value"]
    got = float(line["value"])
    floor = want * (1.0 - tolerance)
    ok = got >= floor
    return ok, (f"{'PASS' if ok else 'FAIL'} {model}: {got:.1f} {line.get('unit', '')} vs baseline {want:.1f} "
                f"(floor {floor:.1f}, {100 * (got / want - 1):+.1f} %)")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", nargs="*", default=None, help="run bench.py for these models instead of reading stdin")
    ap.add_argument("--tolerance", type=float, default=0.05)
    ap.add_argument("--baseline", default=BASELINE)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args(argv)
    with open(a.baseline) as f:
        baseline = json.load(f)
    lines = []
    if a.run:
        for m in a.run:
            out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", m, "--steps", str(a.steps),
                                  "--warmup", "3"], capture_output=True, text=True, check=True).stdout
            lines += [json.loads(x) for x in out.splitlines() if x.startswith("{")]
    else:
        lines = [json.loads(x) for x in sys.stdin.read().splitlines() if x.strip().startswith("{")]
    bad = 0
    for ln in lines:
        ok, msg = check(ln, baseline, a.tolerance)
        print(msg, flush=True)
        bad += not ok
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
