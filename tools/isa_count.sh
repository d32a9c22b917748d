#!/bin/bash
# Static VALU/SALU/VMEM instruction counts and VGPRs of kernels in a --save-temps
# .s file (tuning aid).  Usage: tools/isa_count.sh file.s pattern...
F=$1; shift
for k in "$@"; do
  grep -n "^_Z[A-Za-z0-9_]*${k}[A-Za-z0-9_]*:" "$F" | while IFS=: read st name _; do
    en=$(grep -n "^.Lfunc_end" "$F" | awk -F: -v s="$st" '$1>s{print $1; exit}')
    body=$(sed -n "${st},${en}p" "$F")
    printf "%-70s VALU %4d SALU %4d VMEM %3d vgpr %s\n" "$name" \
      "$(grep -c -E '^\s+v_' <<<"$body")" "$(grep -c -E '^\s+s_' <<<"$body")" \
      "$(grep -c -E '^\s+(global|buffer)_' <<<"$body")" \
      "$(grep "^\s*\.set ${name}\.num_vgpr" "$F" | awk '{print $3}')"
  done
done
