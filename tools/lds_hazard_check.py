"""Lint for the inline-asm LDS reads (fq_lds.h): an asm ds_read's destination is written when the read
RETURNS, but the compiler takes it as written at the asm statement, so any instruction that touches
that register before the lgkmcnt wait retiring the read (a spill store, a copy, a reuse as a
temporary) sees or races the old value.  Scans the device assembly of a kernel in straight-line order
(branches ignored), tracks the outstanding LDS reads in issue order, retires them at s_waitcnt
lgkmcnt(k) (all but the youngest k), and reports every other instruction that reads or writes a
register of a still-outstanding read.  Development tool, not part of the product.

usage: python tools/lds_hazard_check.py file.s [kernel-name-regex]"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def check(lines, name):
    pending = []  # [(line no, dest regs)] in issue order
    bad = []
    for no, raw in lines:
        ins = raw.split(";")[0].strip()
        if not ins or ins.endswith(":") or ins.startswith("."):
            continue
        op = ins.split()[0]
        m = re.match(r"s_waitcnt\b.*lgkmcnt\((\d+)\)", ins)
        if m:
            k = int(m.group(1))
            pending = pending[len(pending) - k:] if k < len(pending) else pending
            if k == 0:
                pending = []
            continue
        if op.startswith("ds_read") or op.startswith("ds_load"):
            operands = ins[len(op):].split(",")
            dst = regs(operands[0])
            srcs = regs(",".join(operands[1:]))
            for pno, pr in pending:
                if pr & (dst | srcs):
                    bad.append((no, pno, ins))
            pending.append((no, dst))
            continue
        if op.startswith("s_load") or op.startswith("s_buffer_load") or op == "s_memrealtime" or op == "s_memtime":
            pending.append((no, set()))  # (counts in lgkmcnt)
            continue
        if op.startswith("ds_write") or op.startswith("ds_store") or op.startswith("ds_"):
            pending.append((no, set()))
        used = regs(ins[len(op):])
        for pno, pr in pending:
            if pr & used:
                bad.append((no, pno, ins))
    for no, pno, ins in bad:
        print(f"{name}: line {no}: `{ins}` touches the destination of the LDS read at line {pno} before its wait")
    return len(bad)


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    text = open(path).read().splitlines()
    n = 0
    cur, body = None, []
    for i, line in enumerate(text, 1):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            if cur and (pat is None or pat.search(cur)):
                n += check(body, cur[:60])
            cur, body = m.group(1), []
            continue
        if cur:
            body.append((i, line))
            if "s_endpgm" in line:
                if pat is None or pat.search(cur):
                    n += check(body, cur[:60])
                cur, body = None, []
    print(f"{n} hazard(s)")
    return 1 if n else 0


if __name__ == "__main__":
    sys.exit(main())
