"""Extract the gfx950 code object(s) embedded in a HIP shared library (clang offload
bundles in its .hip_fatbin section) for disassembly: python scripts/extract_co.py LIB OUTDIR"""
import os
import struct
import sys

lib, out = sys.argv[1], sys.argv[2]
data = open(lib, "rb").read()
magic = b"__CLANG_OFFLOAD_BUNDLE__"
os.makedirs(out, exist_ok=True)
pos, n = 0, 0
while True:
    i = data.find(magic, pos)
    if i < 0:
        break
    (count,) = struct.unpack_from("<Q", data, i + 24)
    p = i + 32
    for _ in range(count):
        off, size, idlen = struct.unpack_from("<QQQ", data, p)
        tid = data[p + 24:p + 24 + idlen].decode()
        p += 24 + idlen
        if "gfx950" in tid and size:
            fn = os.path.join(out, f"co{n}_{tid.replace(':', '_')}.co")
            open(fn, "wb").write(data[i + off:i + off + size])
            print(fn, size)
            n += 1
    pos = i + 1
