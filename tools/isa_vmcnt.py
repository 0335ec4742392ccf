"""List every compiler-placed ``s_waitcnt vmcnt(N > 0)`` of a kernel and the load it
guards, with the inline-asm LDS-DMA pieces issued between the two (DESIGN.md section 5,
the LDS-DMA hazard of the compiler-visible read form; round-5 verdict item 8).

The hypothesis under test: the compiler does not see the inline-asm
``global_load_lds_dwordx4`` pieces as outstanding VMEM operations, so a ``vmcnt(N)`` it
computes for one of its own loads might be "short by the number of pieces in flight".
The listing shows, per wait, the guarded load in the compiler's model (the (N+1)-th most
recent VMEM operation it issued, pieces excluded) and how many pieces were issued between
that load and the wait.  In program order, linear over the code (branches ignored).

    python tools/isa_vmcnt.py <disassembly.s> <kernel-symbol-substring>
"""
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, ln in enumerate(lines) if re.match(r"^[0-9a-f]+ <", ln) and sym in ln)
    end = next((i for i in range(start + 1, len(lines)) if re.match(r"^[0-9a-f]+ <", lines[i])), len(lines))
    ins = []
    for ln in lines[start + 1:end]:
        b = ln.split("//")[0].strip()
        if b and not b.endswith(":"):
            ins.append(b)
    vmem = re.compile(r"^(global_|buffer_|flat_|scratch_)(load|store|atomic)")
    history = []  # (index, text, is_asm_piece)
    print(f"kernel {lines[start].split('<')[1].rstrip('>:')}: {len(ins)} instructions")
    print("wait_index wait | guarded_index guarded_op | asm LDS-DMA pieces between | compiler ops between")
    n_short = 0
    for i, b in enumerate(ins):
        op = b.split()[0]
        if vmem.match(op):
            history.append((i, b, op.startswith("global_load_lds") or " lds" in b))
            continue
        m = re.match(r"s_waitcnt .*vmcnt\((\d+)\)", b)
        if not m or int(m.group(1)) == 0:
            continue
        n = int(m.group(1))
        comp = [h for h in history if not h[2]]
        if len(comp) <= n:
            print(f"{i:6d} {b} | (nothing older than the last {n} compiler ops)")
            continue
        gi, gb, _ = comp[-(n + 1)]
        pieces = sum(1 for h in history if h[2] and h[0] > gi)
        between = sum(1 for h in comp if h[0] > gi)
        # in hardware, the loads younger than the guarded one are the compiler's `between`
        # plus the pieces; vmcnt(n) with n <= that total still covers the guarded load, as
        # loads retire in order -- the wait is short only if a piece retired out of order
        n_short += int(pieces > 0)
        print(f"{i:6d} {b} | {gi:6d} {gb[:60]} | {pieces} | {between}")
    print(f"waits with asm pieces between the guarded load and the wait: {n_short}")


if __name__ == "__main__":
    main()
