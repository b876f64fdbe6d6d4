#!/bin/bash
# Run every built stamp-lab variant (scripts/micro/encode_lab*) once.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for b in scripts/micro/encode_lab scripts/micro/encode_lab_*; do
  case "$b" in *.hip) continue;; esac
  [ -x "$b" ] || continue
  echo "== $b"
  timeout -k 5 60 "$b" || exit $?
done
