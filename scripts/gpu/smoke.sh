#!/bin/bash
# GPU-box job: the driver's round-end smoke() entry point
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")"
