"""Count selected instruction mnemonics in one kernel of a hipcc --save-temps .s file.
usage: isa_count.py FILE.s SYMBOL_SUBSTRING [REGEX]"""
import collections
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
pat = re.compile(sys.argv[3] if len(sys.argv) > 3 else
                 r"\b(v_pk_\w+|v_cvt_\w+|v_add_f32\w*|v_mul_f32\w*|v_add_f16\w*|v_mul_f16\w*|v_fma\w*|"
                 r"global_load_dwordx4|global_store_dwordx4|s_barrier|buffer_inv|buffer_wbl2)\b")
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith(sym) or (sym in l and l.rstrip().endswith(":") and
                                                                      not l.startswith("\t")))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
c = collections.Counter(m.group(1) for l in lines[start:end] for m in [pat.search(l)] if m)
print(lines[start].split(":")[0])
for k, v in sorted(c.items()):
    print(f"  {v:5d} {k}")
