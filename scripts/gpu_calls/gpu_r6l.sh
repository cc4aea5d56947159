#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/dev/lnq8_debug.py 2>&1 | grep -v amdgpu.ids
