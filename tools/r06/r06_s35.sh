#!/bin/bash
# Round-6 session 35: r06_s34 (capsule reciprocal tests + M4 A/B), then every workload line and
# the M5 lean-path A/B (r06_s33).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash tools/r06/r06_s34.sh || exit 1
bash tools/r06/r06_s33.sh
