#!/usr/bin/env python3
"""Per-function totals of a $BT2G_SAMPLE dump (integration/bt2g_prof.cpp).

  python scripts/prof_symbolize.py samples.txt [--top 40]
"""
import argparse
import collections
import os
import subprocess


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def local(path):
    """A GPU box's path of a repository file, mapped into this checkout
    ($BT2G_SYM_BIN=<file>: use that file for the batch server's samples -- the
    binary of the run, when the checkout has been rebuilt since)."""
    alt = os.environ.get("BT2G_SYM_BIN")
    if alt and path.endswith("/bowtie2-align-server-batch"):
        return alt
    if os.path.exists(path) or "/repo/" not in path:
        return path
    return os.path.join(ROOT, path.split("/repo/", 1)[1])


def load_segments(path):
    """(p_offset, p_vaddr, p_filesz) of the executable LOAD segments."""
    out = subprocess.run(["readelf", "-lW", path], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                         text=True).stdout
    segs = []
    for ln in out.splitlines():
        f = ln.split()
        if f and f[0] == "LOAD":
            segs.append((int(f[1], 16), int(f[2], 16), int(f[4], 16)))
    return segs


def to_vaddr(segs, off):
    for o, v, n in segs:
        if o <= off < o + n:
            return off - o + v
    return off


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--role", type=int, default=0, help="only samples of this thread role (1 carrier, "
                    "2 dispatcher), from the (pc, [rsp]) pair table")
    ap.add_argument("--callers-of", default="", help="function name: list the callers of its samples "
                    "(from the (pc, [rsp]) pairs; meaningful for frameless leaves such as syscall wrappers)")
    a = ap.parse_args()
    if a.callers_of:
        return callers(a)
    if a.role:
        return by_role(a)
    by_path = collections.defaultdict(list)
    total = 0
    for ln in open(a.dump):
        if ln.startswith("#"):
            continue
        p, off, c = ln.split()
        by_path[p].append((int(off, 16), int(c)))
        total += int(c)
    funcs = collections.Counter()
    for p, items in by_path.items():
        if p in ("?", "[vdso]") or p.startswith("["):
            for _, c in items:
                funcs[p] += c
            continue
        segs = load_segments(local(p))
        addrs = [hex(to_vaddr(segs, o)) for o, _ in items]
        out = subprocess.run(["addr2line", "-f", "-C", "-e", local(p)] + addrs, stdout=subprocess.PIPE,
                             stderr=subprocess.DEVNULL, text=True).stdout.splitlines()
        names = out[0::2]
        lib = p.rsplit("/", 1)[-1]
        for (o, c), nm in zip(items, names):
            funcs[f"{nm[:110]} [{lib}]"] += c
    print(f"{total} samples")
    for nm, c in funcs.most_common(a.top):
        print(f"{100.0 * c / total:6.2f}%  {c:7d}  {nm}")


def symbolize(pairs):
    """{(path, off): name} for a list of (path, off)."""
    by = collections.defaultdict(set)
    for p, o in pairs:
        by[p].add(o)
    out = {}
    for p, offs in by.items():
        offs = sorted(offs)
        if p == "?" or p.startswith("["):
            for o in offs:
                out[(p, o)] = p
            continue
        segs = load_segments(local(p))
        res = subprocess.run(["addr2line", "-f", "-C", "-e", local(p)] + [hex(to_vaddr(segs, o)) for o in offs],
                             stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True).stdout.splitlines()
        for o, nm in zip(offs, res[0::2]):
            out[(p, o)] = f"{nm[:100]} [{p.rsplit('/', 1)[-1]}]"
    return out


def by_role(a):
    rows = []
    for ln in open(a.dump):
        if ln.startswith("#pair "):
            f = ln.split()
            if len(f) > 6 and int(f[6]) == a.role:
                rows.append(((f[1], int(f[2], 16)), int(f[5])))
    names = symbolize([r[0] for r in rows])
    cnt = collections.Counter()
    for pc, c in rows:
        cnt[names[pc]] += c
    tot = sum(cnt.values())
    print(f"{tot} samples of role {a.role}")
    for nm, c in cnt.most_common(a.top):
        print(f"{100.0 * c / max(tot, 1):6.2f}%  {c:7d}  {nm}")


def callers(a):
    rows = []
    for ln in open(a.dump):
        if ln.startswith("#pair "):
            f = ln.split()
            rows.append(((f[1], int(f[2], 16)), (f[3], int(f[4], 16)), int(f[5]), int(f[6]) if len(f) > 6 else 0))
    names = symbolize([r[0] for r in rows] + [r[1] for r in rows])
    cnt = collections.Counter()
    roles = collections.Counter()
    tot = 0
    for pc, ret, c, role in rows:
        roles[role] += c
        if a.callers_of in names[pc]:
            tag = {1: "carrier", 2: "dispatcher", 9: "carrier (exe caller)", 10: "dispatcher (exe caller)"}
            cnt[f"{tag.get(role, role)}: {names[ret]}"] += c
            tot += c
    print(f"samples by thread role (1 carrier, 2 dispatcher): {dict(roles)}")
    print(f"{tot} samples in {a.callers_of}")
    for nm, c in cnt.most_common(a.top):
        print(f"{c:7d}  {nm}")


if __name__ == "__main__":
    main()
