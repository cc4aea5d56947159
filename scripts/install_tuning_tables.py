"""Copy the tables measured by scripts/gen_tuning_tables.sh (gpurun_out/gemm_tuning_<model>.json)
into replicann_amd/tuning/gemm_<model>.json, sorted and one entry per line (reviewable diffs)."""

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from replicann_amd.tuning import KEYS, canonical  # noqa: E402
MODELS = ["gpt2-small", "gpt2-medium", "gpt2-medium-fp8", "vit-b16", "resnet18"]


def main():
    n = 0
    for m in MODELS:
        src = ROOT / "gpurun_out" / f"gemm_tuning_{m}.json"
        if not src.exists():
            print(f"missing {src}", file=sys.stderr)
            continue
        rows = json.loads(canonical(json.loads(src.read_text())))
        rows.sort(key=lambda r: tuple(r[k] for k in KEYS))
        dst = ROOT / "replicann_amd" / "tuning" / f"gemm_{m}.json"
        dst.write_text("[\n" + ",\n".join(canonical([r])[1:-1] for r in rows) + "\n]\n")
        print(f"{dst.name}: {len(rows)} shapes")
        n += 1
    return 0 if n else 1


if __name__ == "__main__":
    sys.exit(main())
