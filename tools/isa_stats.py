"""Register use and instruction mix of device kernels in a hipcc -save-temps
.s file: python tools/isa_stats.py file.s [name-substring ...]."""
import re
import sys
from collections import Counter


def kernels(text):
    md = text[text.index("amdhsa.kernels"):]
    out = {}
    for ent in md.split("\n  - ")[1:]:
        m = re.search(r"\.name:\s+(\S+)", ent)
        if not m:
            continue
        g = lambda k: int(re.search(r"\." + k + r":\s+(\d+)", ent).group(1)) if re.search(r"\." + k + r":\s+(\d+)", ent) else -1
        out[m.group(1)] = dict(vgpr=g("vgpr_count"), agpr=g("agpr_count"), lds=g("group_segment_fixed_size"),
                               spill=g("vgpr_spill_count"))
    return out


def body(text, name):
    i = text.index("\n" + name + ":")
    j = text.index(".Lfunc_end", i)
    return text[i:j]


def mix(b):
    c = Counter()
    for line in b.splitlines():
        t = line.strip().split()
        if not t or t[0].startswith((";", ".", "_")) or t[0].endswith(":"):
            continue
        op = t[0]
        if op.startswith("v_mfma"):
            c["mfma"] += 1
        elif op.startswith(("v_exp", "v_log", "v_rcp", "v_sqrt", "v_rsq")):
            c["trans"] += 1
        elif op.startswith(("v_accvgpr", "v_mov")):
            c["mov"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("ds_read"):
            c["ds_read"] += 1
        elif op.startswith("ds_write"):
            c["ds_write"] += 1
        elif op.startswith(("global_load", "buffer_load")):
            c["vmem_ld"] += 1
        elif op.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        elif op.startswith("s_barrier"):
            c["barrier"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    return c


if __name__ == "__main__":
    text = open(sys.argv[1]).read()
    subs = sys.argv[2:]
    for name, r in kernels(text).items():
        if subs and not any(s in name for s in subs):
            continue
        print(name[:90], r, dict(mix(body(text, name))))
