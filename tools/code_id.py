#!/usr/bin/env python3
"""The build identity of run-time code objects as sail_jit.cpp codeId computes it: FNV-1a 64 over the .text, .rodata,
.note and .data sections (with their names). Usage: tools/code_id.py FILE.co ... (SAILJIT1 cache files or bare ELF)."""
import struct, sys
def fnv(b, h=14695981039346656037):
    for x in b:
        h ^= x; h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h
def fnvstr(s, h): return fnv(s.encode() + b'\0', h)
def codeid(d):
    shoff, = struct.unpack_from('<Q', d, 0x28); shentsize, shnum, shstrndx = struct.unpack_from('<HHH', d, 0x3a)
    so, ss = struct.unpack_from('<QQ', d, shoff + shstrndx * shentsize + 0x18)
    h = fnv(b'sail-code')
    for k in range(shnum):
        e = shoff + k * shentsize
        no, ty = struct.unpack_from('<II', d, e); off, size = struct.unpack_from('<QQ', d, e + 0x18)
        name = d[so + no: d.index(b'\0', so + no)].decode()
        if name not in ('.text', '.rodata', '.note', '.data'): continue
        h = fnvstr(name, h)
        if ty != 8: h = fnv(d[off:off + size], h)
    return '%016x' % h
for f in sys.argv[1:]:
    d = open(f, 'rb').read()
    if d[:8] == b'SAILJIT1': d = d[32:]
    print(f, codeid(d))
