"""Run-length summary of a kernel's instruction stream in a hipcc `-S` listing: MFMAs (M),
LDS reads (R), LDS writes (Wr), waits (W(...)), barriers (B), global / scratch memory ops by
name.  Shows whether the LDS reads of the next MFMA block are issued ahead of the MFMAs that
would otherwise wait for them.

    python tools/isa_seq.py listing.s 'conv_a_kernelILi64ELi64ELi1ELi0E'
"""
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and pat in l.split(":")[0])
    seq = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        l = l.strip()
        if not l or l.startswith((";", ".")):
            if l.startswith(".LBB"):
                seq.append("|" + l.split(":")[0])
            continue
        t = l.split()[0]
        if t.startswith("v_mfma"):
            k = "M"
        elif t.startswith("ds_read"):
            k = "R"
        elif t.startswith("ds_write"):
            k = "Wr"
        elif t.startswith("s_waitcnt"):
            k = "W(" + l.split(None, 1)[1] + ")"
        elif t.startswith("s_barrier"):
            k = "B"
        elif t.startswith(("scratch", "buffer_", "global_", "s_cbranch")):
            k = t
        else:
            continue
        seq.append(k)
    out, prev, cnt = [], None, 0
    for k in seq + [None]:
        if k == prev:
            cnt += 1
            continue
        if prev:
            out.append("%sx%d" % (prev, cnt) if cnt > 1 else prev)
        prev, cnt = k, 1
    print(" ".join(out))


if __name__ == "__main__":
    main()
