"""Count the VALU instructions of K3's per-node loop in the gfx950 assembly.

Used for the VALU-issue roofline of the pod x node kernel (bench.py): one loop
iteration evaluates one node for the 64 pods of a wave.  All blocks of the loop
are counted (divergent blocks included), so this is the per-iteration issue
cost when every path is taken.
"""
import json
import re
import sys


def loop_valu(asm: str, func_pat: str):
    m = re.search(r"^(" + func_pat + r"):", asm, re.M)
    if not m:
        raise SystemExit(f"function {func_pat} not found")
    body = asm[m.end(): asm.index("s_endpgm", m.end())]
    counts, in_loop = {"valu": 0, "salu": 0, "smem": 0, "vmem": 0}, False
    # drop loop blocks that call the exact (rare) path: count the fast path
    blocks, cur = [], []
    for line in body.splitlines():
        t = line.strip()
        if (t.startswith(".LBB") or t.startswith("; %bb.")) and cur:
            blocks.append(cur)
            cur = []
        cur.append(line)
    blocks.append(cur)
    body = "\n".join(l for b in blocks if not any("s_swappc" in x for x in b) for l in b)
    for line in body.splitlines():
        t = line.strip()
        if t.startswith(".LBB") or t.startswith("; %bb."):
            in_loop = "Loop: Header=" in t or "Inner Loop Header" in t
            continue
        if "Inner Loop Header" in t or "in Loop: Header" in t:
            in_loop = True
            continue
        if not in_loop or not t or t.startswith(";") or t.startswith("."):
            continue
        op = t.split()[0]
        if op.startswith("v_"):
            counts["valu"] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            counts["smem"] += 1
        elif op.startswith("s_"):
            counts["salu"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            counts["vmem"] += 1
    return counts


if __name__ == "__main__":
    asm = open(sys.argv[1]).read()
    out = {"kernel": "k3_eval<4,6,false,V>", "variants": {}}
    for v, nodes in ((0, 1), (1, 1), (2, 2), (3, 1), (4, 1)):
        c = loop_valu(asm, r"_ZN5crane7k3_evalILi4ELi6ELb0ELi%dEEEv\S*" % v)
        out["variants"][str(v)] = {"valu_per_node": c["valu"] / nodes, "salu_per_node": c["salu"] / nodes,
                                   "smem_per_node": c["smem"] / nodes, "vmem_per_node": c["vmem"] / nodes}
    out["default_variant"] = 4  # kernels.hip k3_variant() default
    out["valu_per_node_iter"] = out["variants"]["4"]["valu_per_node"]
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(out)
