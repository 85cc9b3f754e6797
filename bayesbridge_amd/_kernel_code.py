"""Identity of a kernel's machine code in BayesBridge.so, for the measurement evidence.

A committed profile (kernel durations, PMC traffic, VALU instruction counts) describes the
kernel it measured; bench.py may use it for a later build only if that kernel's gfx950 code is
the same.  `code_shas()` reads the clang offload bundles embedded in the library (one per HIP
translation unit), parses each gfx950 ELF code object and hashes, per kernel, its code bytes
together with its kernel descriptor (`<name>.kd`: register counts, LDS size, launch flags;
its entry offset, which only locates the code, left out).
A code object's out-of-line device functions (callees) are folded into the identity of each of
its kernels.  Two builds whose hashes agree for a kernel run the same instructions with the same
resources; any change of the kernel's source, of an inlined or called helper or of the
compiler changes it.

Pure host code (no GPU, no HIP calls): usable on the CPU container and on the GPU box.
"""
from __future__ import annotations

import hashlib
import os
import re
import struct

from . import _build

_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_CACHE: dict = {}


def _bundles(blob: bytes):
    """(triple, bytes) of every entry of every uncompressed offload bundle in blob."""
    pos = 0
    while True:
        i = blob.find(_BUNDLE_MAGIC, pos)
        if i < 0:
            return
        (n,) = struct.unpack_from("<Q", blob, i + 24)
        off = i + 32
        for _ in range(n):
            eo, es, ts = struct.unpack_from("<QQQ", blob, off)
            triple = blob[off + 24:off + 24 + ts].decode("ascii", "replace")
            off += 24 + ts
            yield triple, blob[i + eo:i + eo + es]
        pos = i + len(_BUNDLE_MAGIC)


def _elf_symbols(elf: bytes, funcs: dict | None = None):
    """{name: (bytes of the symbol)} for the FUNC and OBJECT symbols of an ELF64 code object;
    `funcs`, if given, also receives the FUNC symbols alone."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        return {}
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, _ = struct.unpack_from("<HHH", elf, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + k * shentsize) for k in range(shnum)]
    out = {}
    for sec in secs:
        if sec[1] != 2:  # SHT_SYMTAB
            continue
        _, _, _, _, off, size, link, _, _, ent = sec
        stroff = secs[link][4]
        for k in range(size // ent):
            st_name, st_info, _, shndx, value, ssize = struct.unpack_from(
                "<IBBHQQ", elf, off + k * ent)
            if (st_info & 0xF) not in (1, 2) or shndx == 0 or shndx >= len(secs) or ssize == 0:
                continue
            end = elf.index(b"\0", stroff + st_name)
            name = elf[stroff + st_name:end].decode("ascii", "replace")
            tsec = secs[shndx]
            start = tsec[4] + (value - tsec[3])
            out[name] = elf[start:start + ssize]
            if funcs is not None and (st_info & 0xF) == 2:
                funcs[name] = out[name]
    return out


def code_shas(so_path: str | None = None) -> dict:
    """{mangled kernel name: sha256[:16] of its code bytes + its .kd descriptor} for every
    gfx950 kernel in the library."""
    so_path = so_path or _build.SO_PATH
    key = (so_path, os.path.getmtime(so_path))
    if key in _CACHE:
        return _CACHE[key]
    blob = open(so_path, "rb").read()
    out = {}
    for triple, elf in _bundles(blob):
        if "gfx950" not in triple:
            continue
        funcs: dict = {}
        syms = _elf_symbols(elf, funcs)
        # out-of-line device functions of this code object (no .kd: not kernels), e.g. the
        # __noinline__ sampler bodies the NI lambda variants call: their code is part of every
        # kernel's identity in the code object (which kernel calls which is not resolved), so
        # an edit of a callee retires the evidence of its callers
        callees = sorted(n for n in funcs if not n.endswith(".kd") and n + ".kd" not in syms)
        cdig = b""
        if callees:
            h = hashlib.sha256()
            for n in callees:
                h.update(n.encode() + b"\0" + funcs[n])
            cdig = b"|" + h.digest()
        for name, code in syms.items():
            if name.endswith(".kd"):
                continue
            kd = syms.get(name + ".kd")
            if kd is None:
                continue  # a device function, not a kernel
            # the descriptor's kernel_code_entry_byte_offset (bytes 16-23) is the distance to
            # the code, which moves with the layout of the code object: not part of identity
            kd = kd[:16] + bytes(8) + kd[24:]
            out[name] = hashlib.sha256(code + b"|" + kd + cdig).hexdigest()[:16]
    _CACHE[key] = out
    return out


def mangled_prefix(instance: str) -> str:
    """bb::k_lambda_xu<8, 8> -> _ZN2bb11k_lambda_xuILi8ELi8EEEv (int / bool template
    arguments; a template kernel's mangling carries its void return type); bb::k_pre ->
    _ZN2bb5k_preE."""
    m = re.match(r"bb::(\w+)(?:<(.*)>)?$", instance.strip())
    if not m:
        raise ValueError(f"not a bb:: kernel instance: {instance!r}")
    base, args = m.group(1), m.group(2)
    s = f"_ZN2bb{len(base)}{base}"
    if args is None:
        return s + "E"
    s += "I"
    for a in (x.strip() for x in args.split(",")):
        s += {"true": "Lb1E", "false": "Lb0E"}.get(a, f"Li{a}E")
    return s + "EEv"


def code_sha(instance: str, so_path: str | None = None) -> str | None:
    """Code identity of one kernel instance named as rocprofv3 / bb_kernel_instance name it
    ("bb::k_eapply<8, 0>"); None if the library holds no unique kernel of that name."""
    pre = mangled_prefix(instance)
    hits = [v for k, v in code_shas(so_path).items() if k.startswith(pre)]
    return hits[0] if len(hits) == 1 else None


def annotate(kernels: dict, shas: dict) -> int:
    """Add "code_sha" to every bb:: entry of a profile's {instance: entry} map from shas
    (code_shas() of the library that was profiled); returns the number annotated."""
    k = 0
    for name, entry in kernels.items():
        if not name.startswith("bb::") or not isinstance(entry, dict):
            continue
        try:
            pre = mangled_prefix(name)
        except ValueError:
            continue
        hits = [v for m, v in shas.items() if m.startswith(pre)]
        if len(hits) == 1:
            entry["code_sha"] = hits[0]
            k += 1
    return k


if __name__ == "__main__":  # the code identities of this tree's library, as JSON
    import json
    import sys

    json.dump(code_shas(sys.argv[1] if len(sys.argv) > 1 else None), sys.stdout, indent=0)
