#!/usr/bin/env python3
"""Per-kernel scratch (private segment) and LDS sizes of the gfx950 code
object inside a built library, read from the kernel descriptors (`<kernel>.kd`
symbols: group_segment_fixed_size at byte 0, private_segment_fixed_size at
byte 4).  A kernel with a scratch segment gets its waves dispatched later
(DESIGN section 6); the per-merge kernels must have none.

usage: tools/kernel_scratch.py [lib.so]   (prints kernel, LDS bytes, scratch bytes/lane)
"""
import struct
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(blob):
    """(triple, ELF bytes) of every entry of every offload bundle in blob"""
    pos = blob.find(MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", blob, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            yield triple, blob[pos + off:pos + off + size]
        pos = blob.find(MAGIC, pos + 1)


def kernel_descriptors(elf):
    """{kernel name: (lds bytes, scratch bytes per lane)} from the .kd symbols"""
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    out = {}
    for s in secs:
        if s[1] != 2:  # SHT_SYMTAB
            continue
        strtab = secs[s[6]]
        for k in range(s[5] // 24):
            name_off, info, other, shndx, value, size = struct.unpack_from("<IBBHQQ", elf, s[4] + k * 24)
            end = elf.index(b"\0", strtab[4] + name_off)
            name = elf[strtab[4] + name_off:end].decode()
            if not name.endswith(".kd") or shndx == 0 or shndx >= len(secs):
                continue
            sec = secs[shndx]
            fo = sec[4] + (value - sec[3])  # file offset of the descriptor
            lds, scratch = struct.unpack_from("<II", elf, fo)
            out[name[:-3]] = (lds, scratch)
    return out


def scan(path):
    blob = open(path, "rb").read()
    res = {}
    for triple, elf in code_objects(blob):
        if "gfx950" in triple and elf[:4] == b"\x7fELF":
            res.update(kernel_descriptors(elf))
    return res


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else "llmtokenizer_amd/libbpe_amd.so"
    for k, (lds, scr) in sorted(scan(lib).items()):
        print(f"{k:90s} lds {lds:7d} scratch {scr:5d}")
