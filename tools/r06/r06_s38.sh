#!/bin/bash
# Round-6 session 38: r06_s37 (plain KParams box, M1) then r06_s36 (coop-lane thresholds, M2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash tools/r06/r06_s37.sh || exit 1
bash tools/r06/r06_s36.sh
