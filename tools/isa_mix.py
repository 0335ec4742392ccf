"""Static instruction mix of the loops of a kernel (diagnostic): every backward branch of
the kernel's disassembly delimits a loop; prints, per loop of at least ``--min`` instructions,
the counts of MFMA, transcendental VALU, other VALU, LDS, VMEM, waits and SALU.

    /opt/rocm/lib/llvm/bin/llvm-objdump -d --mcpu=gfx950 <code object> > k.s
    python tools/isa_mix.py k.s kp_attn3ILi13ELi2E
"""
import argparse
import collections
import re

TRANS = ("v_exp_f32", "v_rcp_f32", "v_log_f32", "v_rsq_f32", "v_sqrt_f32", "v_rcp_iflag_f32", "v_exp_f64",
         "v_rcp_f64", "v_sin", "v_cos")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("disasm")
    ap.add_argument("symbol")
    ap.add_argument("--min", type=int, default=300)
    a = ap.parse_args()
    lines = open(a.disasm).read().split("\n")
    st = next(i for i, ln in enumerate(lines) if re.match(r"^[0-9a-f]+ <", ln) and a.symbol in ln)
    en = next((i for i in range(st + 1, len(lines)) if re.match(r"^[0-9a-f]+ <", lines[i])), len(lines))
    ins = []
    for ln in lines[st + 1:en]:
        m = re.match(r"\s+([a-z_0-9]+)(.*?)//\s*([0-9A-F]+):", ln)
        if m:
            ins.append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
    print(lines[st].strip())
    for addr, op, args in ins:
        if not (op.startswith("s_cbranch") or op == "s_branch"):
            continue
        try:
            off = int(args.split()[0])
        except ValueError:
            continue
        if off >= 32768:
            off -= 65536
        tgt = addr + 4 + 4 * off
        if tgt >= addr:
            continue
        body = [o for x, o, _ in ins if tgt <= x <= addr]
        if len(body) < a.min:
            continue
        c = collections.Counter()
        for o in body:
            if o.startswith("v_mfma"):
                c["mfma"] += 1
            elif o.startswith(TRANS):
                c["valu_trans"] += 1
            elif o.startswith("v_"):
                c["valu"] += 1
            elif o.startswith("ds_"):
                c["lds:" + o] += 1
            elif o.startswith(("global_", "buffer_")):
                c["vmem"] += 1
            elif o.startswith(("s_waitcnt", "s_nop", "s_barrier")):
                c["wait/nop/barrier"] += 1
            elif o.startswith("s_"):
                c["salu"] += 1
        print(f"loop {tgt:#x}..{addr:#x} ({len(body)} instructions): {dict(sorted(c.items()))}")


if __name__ == "__main__":
    main()
