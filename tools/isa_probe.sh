#!/bin/bash
# Which packed min/max forms gfx950 has (DESIGN §11.3's n = 4 epilogue floor): each line assembled alone with
# the ROCm LLVM assembler for gfx950; "NO" = the assembler rejects the instruction for this target.
# usage: tools/isa_probe.sh   (CPU only: no GPU needed)
MC=/opt/rocm/lib/llvm/bin/llvm-mc
t=$(mktemp -d)
while read -r ins; do
  echo "$ins" > "$t/one.s"
  if "$MC" -arch=amdgcn -mcpu=gfx950 "$t/one.s" > /dev/null 2>&1; then echo "OK  $ins"; else echo "NO  $ins"; fi
done <<'LIST'
v_min3_f32 v0, v1, v2, v3
v_min3_u32 v0, v1, v2, v3
v_minimum3_f32 v0, v1, v2, v3
v_pk_min_f32 v[0:1], v[2:3], v[4:5]
v_pk_max_f32 v[0:1], v[2:3], v[4:5]
v_pk_add_f32 v[0:1], v[2:3], v[4:5]
v_pk_min_f16 v0, v1, v2
v_pk_minimum3_f16 v0, v1, v2, v3
v_pk_min_u16 v0, v1, v2
v_pk_min_i16 v0, v1, v2
LIST
rm -rf "$t"
