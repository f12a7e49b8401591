#!/bin/bash
# Regenerates the libhdf5-written cooler fixtures and their libhdf5 listings
# (build container only: needs the HDF5 1.10 library + headers in /opt/conda;
# h5cc there names a conda compiler that is absent, so gcc is called directly).
# usage: tests/golden/make_h5_fixtures.sh [outdir]   (default: tests/golden)
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="${1:-$HERE}"
H5="${HDF5_PREFIX:-/opt/conda}"
BIN="$(mktemp -d)/make_h5_fixtures"
gcc -O2 -Wall -I"$H5/include" -o "$BIN" "$HERE/make_h5_fixtures.c" -L"$H5/lib" -Wl,-rpath,"$H5/lib" -lhdf5
"$BIN" gen "$OUT"
for f in cooler_earliest cooler_latest; do
  "$BIN" dump "$OUT/$f.cool" | LC_ALL=C sort > "$OUT/$f.listing.txt"
done
rm -f "$BIN"
