#!/bin/bash
# Device-ISA comparison of two builds' kernel objects (round 6): unbundles the gfx950 code object of every
# build/obj/dprf_kernels_*.o in OBJ_A and OBJ_B and diffs their disassembly.  An empty diff means the kernels of
# the two builds are the same machine code, so a source change (e.g. removing dead A/B variants) cannot move a
# bench number.   usage: tools/isa_diff.sh OBJ_A OBJ_B
set -euo pipefail
A=${1:?object dir A}; B=${2:?object dir B}
L=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
rc=0
for f in "$A"/dprf_kernels_*.o; do
    o=$(basename "$f" .o)
    for side in A B; do
        d=$([ $side = A ] && echo "$A" || echo "$B")
        $L/llvm-objcopy --dump-section .hip_fatbin="$T/$side.fb" "$d/$o.o" "$T/junk.o"
        tgt=$($L/clang-offload-bundler --list --type=o --input="$T/$side.fb" | grep gfx950)
        $L/clang-offload-bundler --type=o --targets="$tgt" --input="$T/$side.fb" --output="$T/$side.co" --unbundle
        $L/llvm-objdump -d --no-show-raw-insn "$T/$side.co" | grep -v "file format" > "$T/$o.$side.s"
    done
    n=$(diff "$T/$o.A.s" "$T/$o.B.s" | wc -l || true)
    echo "$o: $(wc -l < "$T/$o.A.s") / $(wc -l < "$T/$o.B.s") lines, diff $n"
    [ "$n" = 0 ] || rc=1
done
rm -rf "$T"
exit $rc
