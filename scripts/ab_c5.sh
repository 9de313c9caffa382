#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
while read -r line; do
  [ -z "$line" ] && continue
  echo "== [$line] $(env $line timeout -k 10 120 python scripts/probe_c5.py 2>&1 | tail -1)"
done <<< "$AB"
