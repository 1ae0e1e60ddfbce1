#!/bin/bash
# Build libfheregex.so of a git revision (A/B baseline) into fhe-regex_amd/build/exp/lib_NAME.so:
#   tools/build_rev.sh NAME REV [-DFOO=1 ...]
set -e
cd "$(dirname "$0")/.."
name=$1; rev=$2; shift 2
tmp=$(mktemp -d /tmp/fr_rev.XXXXXX)
git archive "$rev" fhe-regex_amd include | tar -x -C "$tmp"
make -s -C "$tmp/fhe-regex_amd" -j8 HIPFLAGS_EXTRA="$*" >/dev/null
mkdir -p fhe-regex_amd/build/exp
cp "$tmp/fhe-regex_amd/libfheregex.so" "fhe-regex_amd/build/exp/lib_$name.so"
rm -rf "$tmp"
echo "built fhe-regex_amd/build/exp/lib_$name.so ($rev)"
