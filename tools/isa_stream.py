"""Compressed instruction stream of one kernel's loops in a hipcc -S file:
   python tools/isa_stream.py file.s name-substring [--all]
One letter per instruction: M mfma, r ds_read, t ds_read_b64_tr, w ds_write,
E v_exp, v other VALU, G global load, S global store, s SALU, n s_nop,
|x| s_waitcnt, #BAR# s_barrier.  Prints each loop body (a block ending in a
backward branch) unless --all (the whole kernel)."""
import re
import sys


def body(text, sub):
    names = re.findall(r"^(\S*" + re.escape(sub) + r"\S*):", text, re.M)
    names = [n for n in names if not n.startswith(".")]
    if not names:
        sys.exit(f"no kernel matching {sub}")
    name = names[0]
    i = text.index("\n" + name + ":")
    j = text.index(".Lfunc_end", i)
    return name, text[i:j].splitlines()


def code(line):
    s = line.strip()
    if not s or s.startswith((";", ".")) or s.endswith(":"):
        return None
    op = s.split()[0]
    if op.startswith("v_mfma"):
        return "M"
    if op.startswith("ds_read_b64_tr"):
        return "t"
    if op.startswith("ds_read"):
        return "r"
    if op.startswith("ds_write"):
        return "w"
    if op.startswith("v_exp"):
        return "E"
    if op.startswith(("global_load", "buffer_load")):
        return "G"
    if op.startswith(("global_store", "buffer_store")):
        return "S"
    if op.startswith("s_waitcnt"):
        return "|" + s.split()[1] + "|"
    if op.startswith("s_barrier"):
        return "#BAR#"
    if op.startswith("s_nop"):
        return "n"
    if op.startswith("v_"):
        return "v"
    if op.startswith("s_"):
        return "s"
    return op


def main():
    name, lines = body(open(sys.argv[1]).read(), sys.argv[2])
    print(name)
    if "--all" in sys.argv:
        print(" ".join(c for c in map(code, lines) if c))
        return
    labels = {}
    for k, l in enumerate(lines):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = k
    for k, l in enumerate(lines):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\S+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < k:
            seg = [c for c in map(code, lines[labels[m.group(1)]:k + 1]) if c]
            print(f"loop {m.group(1)}: {len(seg)} instr, {seg.count('M')} mfma, "
                  f"{sum(c in 'vE' for c in seg)} valu, {seg.count('r') + seg.count('t')} ds_read")
            print(" ".join(seg))


if __name__ == "__main__":
    main()
