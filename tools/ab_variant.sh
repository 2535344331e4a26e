#!/bin/bash
# Export the working tree (HEAD + uncommitted diff) into ab/<name>/, apply the python
# substitutions in $SUBS (a file of "path<TAB>old<TAB>new" lines, \n escapes allowed) and build it,
# for same-box A/B runs (tools/ab_dirs.py, TREE=... tools/rocprof_flags.sh).
# Usage: tools/ab_variant.sh name [subs-file]
set -e
cd "$(dirname "$0")/.."
name=$1; subs=$2
rm -rf "ab/$name" && mkdir -p "ab/$name"
git archive HEAD | tar -x -C "ab/$name"
git diff HEAD > "ab/$name.patch"
(cd "ab/$name" && { [ -s "../$name.patch" ] && patch -s -p1 < "../$name.patch" || true; })
if [ -n "$subs" ]; then
  python3 - "ab/$name" "$subs" <<'PY'
import sys
root, subs = sys.argv[1], sys.argv[2]
for line in open(subs):
    line = line.rstrip('\n')
    if not line.strip():
        continue
    path, old, new = line.split('\t')
    old, new = old.replace('\\n', '\n'), new.replace('\\n', '\n')
    p = f'{root}/{path}'
    s = open(p).read()
    assert old in s, (path, old)
    open(p, 'w').write(s.replace(old, new))
PY
fi
(cd "ab/$name" && python3 -c "from kaolin_amd import _build; _build.build()")
echo "ab/$name ready"
