#!/bin/bash
# weaken.sh IN.o OUT.o SYM... -- copy IN.o to OUT.o with each SYM made weak and a
# global alias bt2g_real_SYM at the same address (objcopy): the binding's
# strong definition of SYM then receives the object's own calls to it
# (they go through R_X86_64_PLT32 relocations against the symbol, -fPIC), and
# can still call the reference's definition through the alias.
set -e
in=$1; out=$2; shift 2
args=()
for s in "$@"; do
  line=$(objdump -t "$in" | awk -v s="$s" '$NF==s')
  [ -n "$line" ] || { echo "weaken.sh: $s not in $in" >&2; exit 1; }
  addr=$(echo "$line" | awk '{print $1}')
  sec=$(echo "$line" | awk '{print $4}')
  args+=(--weaken-symbol="$s" --add-symbol "bt2g_real_$s=$sec:0x$addr,global,function")
done
objcopy "${args[@]}" "$in" "$out"
