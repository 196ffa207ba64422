#!/bin/bash
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_ab_tnshare.sh
bash scripts/gpu_pmc_attn3.sh
