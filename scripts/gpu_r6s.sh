#!/bin/bash
# Round 6: host profile of the CFed and MPS rounds (cProfile of 50 enqueued rounds)
source "$(dirname "$0")/gpu_step.sh"
TAILN=0 step hp_cfed128 300 python scripts/host_profile.py cfed128 --rounds 50
TAILN=0 step hp_mps 300 python scripts/host_profile.py vqc48q_mps64 --rounds 50
