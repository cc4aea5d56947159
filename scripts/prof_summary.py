"""Per-step kernel breakdown from a rocprofv3 ``--kernel-trace`` CSV
(thin wrapper over ``replicann_amd.utils.profiling``).

    python scripts/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps 3
"""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from replicann_amd.utils.profiling import main  # noqa: E402

if __name__ == "__main__":
    main(["trace", *sys.argv[1:]])
