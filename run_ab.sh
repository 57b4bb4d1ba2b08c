#!/bin/bash
# process-isolated interleaved A/B: tools/ab.py --spawn
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 tools/ab.py --spawn ${SPAWN:-3} --rounds 4 "$@"
