#!/bin/bash
# Builds libtsdbhip.so of git revision $1 (default HEAD) as
# opentsdb_amd/libtsdbhip_old.so, for same-box A/B runs (tools/gpu/ab.sh).
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" opentsdb_amd/csrc include | tar -x -C "$T"
make -s -C "$T/opentsdb_amd/csrc" OUT="$ROOT/opentsdb_amd/libtsdbhip_old.so"
rm -rf "$T"
