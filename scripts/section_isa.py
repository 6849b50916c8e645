"""Static instruction counts between the section markers of a PT_MARKS build.

usage: python scripts/section_isa.py build/pt_kernel_marks.s [kernel-substring]
Prints, for each stretch of the kernel's assembly between two `; @mark` comments (in
file order), the VALU / SALU / LDS / VMEM instruction counts and the VALU forms that
dual-issue on the second port (f32 add/sub/mul, integer add/and/mov: DESIGN.md §5).
Static counts: rarely taken branches inside a stretch are included.
"""
import re
import sys

path = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else "ILb1ELb0ELi8ELb1EE"
s = open(path).read()
starts = [m.start() for m in re.finditer(r"^(?:_Z\S+|pt_trace_flat_rtc):", s, re.M)]
body = None
for i, st in enumerate(starts):
    name = s[st:s.index(":", st)]
    if want in name:
        end = s.find(".Lfunc_end", st)
        body = s[st:end]
        break
if body is None:
    sys.exit("kernel not found")
DUAL = re.compile(r"^v_(add|sub|subrev|mul)_f32|^v_(add|sub|subrev)_u32|^v_and_b32|^v_mov_b32|^v_or_b32")
cur, rows, order = "entry", {}, []
def row(n):
    if n not in rows:
        rows[n] = dict(valu=0, dual=0, salu=0, lds=0, vmem=0)
        order.append(n)
    return rows[n]
for line in body.split("\n"):
    t = line.strip()
    m = re.match(r";\s*@mark\s+(\S+)", t)
    if m:
        cur = m.group(1)
        continue
    if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
        continue
    op = t.split()[0]
    r = row(cur)
    if op.startswith("v_"):
        r["valu"] += 1
        if DUAL.match(op):
            r["dual"] += 1
    elif op.startswith("s_"):
        r["salu"] += 1
    elif op.startswith("ds_"):
        r["lds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        r["vmem"] += 1
print(f"{'after mark':12s} {'valu':>6s} {'dual':>6s} {'salu':>6s} {'lds':>5s} {'vmem':>5s}")
for n in order:
    r = rows[n]
    print(f"{n:12s} {r['valu']:6d} {r['dual']:6d} {r['salu']:6d} {r['lds']:5d} {r['vmem']:5d}")
