"""Scan gfx950 assembly (hipcc --save-temps .s) for a VMEM store whose data
VGPRs an instruction within the next N instructions overwrites -- the store
data WAR window the round-6 gemm_wsp investigation found (DESIGN.md section 8,
round 6).  python tools/lab/store_war_scan.py file.s [N]"""
import re
import sys

STORE = re.compile(r"^\s*(buffer_store_dword\w*|global_store_dword\w*|flat_store_dword\w*)\s+(\S+?),")
VREG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)")


def regs(tok):
    m = VREG.fullmatch(tok.strip())
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def main(path, n=4):
    lines = [ln.rstrip("\n") for ln in open(path)]
    fn = None
    hits = 0
    for i, ln in enumerate(lines):
        if re.match(r"^_Z\S+:", ln):
            fn = ln.split(":")[0]
        m = STORE.match(ln)
        if not m:
            continue
        data = regs(m.group(2))
        if len(data) <= 2:   # the documented hazard is for stores of more than 64 bits
            continue
        k = 0
        for j in range(i + 1, len(lines)):
            t = lines[j].strip()
            if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
                continue
            k += 1
            if k > n:
                break
            if t.startswith("s_nop"):
                k += int(t.split()[1])
                continue
            op = t.split()[0]
            if op.startswith("v_") and "mfma" not in op:
                dst = t.split()[1].rstrip(",")
                if regs(dst) & data:
                    hits += 1
                    print(f"{path}:{i + 1}: {fn}: '{t}' {k} instr after '{ln.strip()}'")
                    break
    print(f"{hits} store-data WAR windows within {n} instructions")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
