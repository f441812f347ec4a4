#!/usr/bin/env python3
"""Static ISA attribution of one kernel of /tmp/isa/trace_g.s (tools/isa.sh): instructions per source line,
optionally only those whose opcode matches a regex, and the opcode histogram.
  python tools/isa_attr.py KERNEL [OPCODE_REGEX] [--hist] [--top N]"""
import collections
import re
import sys


def kernel_lines(path, name):
    lines = open(path).read().split('\n')
    out, on = [], False
    for l in lines:
        m = re.match(r'^[0-9a-f]+ <(\S+)>:', l)
        if m:
            on = m.group(1) == name
            continue
        if on:
            out.append(l)
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    top = 40
    if '--top' in sys.argv:
        top = int(sys.argv[sys.argv.index('--top') + 1])
        args = [a for a in args if a != str(top)]
    name, pat = args[0], (args[1] if len(args) > 1 else None)
    cur, cnt, hist = '?', collections.Counter(), collections.Counter()
    for l in kernel_lines('/tmp/isa/trace_g.s', name):
        m = re.match(r'; (\S+):(\d+)', l)
        if m:
            cur = m.group(1).split('/')[-1] + ':' + m.group(2)
            continue
        s = l.strip()
        if not s or s.startswith(';') or s.endswith(':'):
            continue
        op = s.split()[0]
        if pat is None or re.search(pat, op):
            cnt[cur] += 1
            hist[op] += 1
    tot = sum(cnt.values())
    print(f"{name}: {tot} instructions" + (f" matching {pat}" if pat else ""))
    if '--hist' in sys.argv:
        for k, v in hist.most_common(top):
            print(f"{v:7d} {k}")
    else:
        for k, v in cnt.most_common(top):
            print(f"{v:7d} {k}")


if __name__ == '__main__':
    main()
