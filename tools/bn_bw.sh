#!/bin/bash
# bn_bw.py under a few grid-size settings
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for st in "" "$@"; do
  echo "== $st"
  env $st timeout -k 10 120 python3 tools/bn_bw.py 2>/dev/null || exit 1
done
