#!/bin/bash
# round 3 baseline: headline bench + kernel-trace profile of the GPT-2-small step
bash scripts/gpu_steps.sh bench prof
