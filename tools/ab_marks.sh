#!/bin/bash
# Block timing of the split train kernel with two stamps per build (MHPPO_MARK_MASK), so each block
# is timed with the rest of the tile unperturbed by the other stamps.
#   build: bash tools/ab_marks.sh build <prefix> [csrc dir]   -> build_ab/<prefix>_m<a><b>/libmhppo.so
#   run:   bash tools/ab_marks.sh run <prefix>                 (GPU; prints the end-mark slot per build)
set -o pipefail
PAIRS="1:2 2:3 3:4 4:5 5:6 6:7 7:8 8:9 9:1"
if [ "$1" = build ]; then
  SRC=${3:-mh-ppo_amd/csrc}
  for p in $PAIRS; do
    a=${p%:*}; b=${p#*:}; m=$(( (1 << a) | (1 << b) ))
    make -s -C $SRC -j2 BUILD=$PWD/build_ab/$2_m$a$b/obj OUT=$PWD/build_ab/$2_m$a$b/libmhppo.so \
      EXTRA="-DMHPPO_TIMING -DMHPPO_MARK_MASK=$m" > /dev/null 2>&1 &
  done
  wait
  ls build_ab | grep "^$2_m" | wc -l
else
  for p in $PAIRS; do
    a=${p%:*}; b=${p#*:}
    X3_PHASES_ALL=1 MHPPO_LIB=build_ab/$2_m$a$b/libmhppo.so timeout -k 10 120 python tools/x3_phases.py > /tmp/m.txt 2>&1 || { cat /tmp/m.txt; exit 1; }
    python3 - $a $b <<'PY'
import re, sys
a, b = sys.argv[1], sys.argv[2]
t = open('/tmp/m.txt').read()
for part in t.split('kind ')[1:]:
    kind = part[0]
    tot = re.search(r'(\d+) stamped cycles/tile', part).group(1)
    m = re.search(r'slot ' + b + r'\s+[\d.]+ %\s+\(\s*(\d+) cycles/tile', part)
    print(f"kind {kind} block {a}->{b}: {m.group(1) if m else '?'} cycles/tile (stamped total {tot})")
PY
  done
fi
