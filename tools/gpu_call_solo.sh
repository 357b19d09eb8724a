#!/bin/bash
# one GPU call: per-rank solo time of the sharded dense solve, b4 vs one-wave tier kernel
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh "400:solo_variants:python -u tools/solo_variants.py 8"
