#!/bin/bash
# Export a git revision into ab/<name>/ and build its library there (on the CPU host), so that
# tools/ab_dirs.py can compare it with the working tree on one GPU box.
# Usage: tools/ab_prepare.sh REV [name]
set -e
cd "$(dirname "$0")/.."
rev=$1; name=${2:-$1}
rm -rf "ab/$name" && mkdir -p "ab/$name"
git archive "$rev" | tar -x -C "ab/$name"
(cd "ab/$name" && python3 -c "from kaolin_amd import _build; _build.build()")
echo "ab/$name ready"
