"""SNP-dict I/O that executes nothing from the file.

The reference caches its parsed VCF (`make_data_dict_vcf`, twoDSFS_class.py:36-138)
as a bz2-compressed pickle (twoDSFS.py:504-510, loaded at twoDSFS_class.py:1918-1919;
shipped example: data/chr1.pkl.bz2).  Unpickling runs arbitrary code, so this module
reads such caches with a *data-only* opcode interpreter: dicts, lists, tuples, str,
int, float, bool and None are rebuilt; any opcode that could import or call
(GLOBAL, STACK_GLOBAL, REDUCE, BUILD, NEWOBJ, INST, OBJ, PERSID, EXT*) is refused.

It also provides the packed, pickle-free cache format used by this framework
(`save_packed` / `load_packed`: numpy .npz with allow_pickle=False).
"""
from __future__ import annotations

import bz2
import gzip
import struct

import numpy as np

__all__ = ["safe_load_pickle_bytes", "load_snp_dict_pkl", "save_packed", "load_packed"]


class RefusedOpcode(ValueError):
    pass


_MARK = object()


def safe_load_pickle_bytes(data: bytes):
    """Rebuild a pickle made only of plain-data opcodes (protocol 0-5 binary forms)."""
    stack: list = []
    memo: dict = {}
    i = 0
    n = len(data)
    unpack_from = struct.unpack_from
    while i < n:
        op = data[i]
        i += 1
        if op == 0x8C:  # SHORT_BINUNICODE
            ln = data[i]
            stack.append(data[i + 1:i + 1 + ln].decode("utf-8", "surrogatepass"))
            i += 1 + ln
        elif op == 0x94:  # MEMOIZE
            memo[len(memo)] = stack[-1]
        elif op == 0x68:  # 'h' BINGET
            stack.append(memo[data[i]])
            i += 1
        elif op == 0x6A:  # 'j' LONG_BINGET
            stack.append(memo[unpack_from("<I", data, i)[0]])
            i += 4
        elif op == 0x4B:  # 'K' BININT1
            stack.append(data[i])
            i += 1
        elif op == 0x4D:  # 'M' BININT2
            stack.append(unpack_from("<H", data, i)[0])
            i += 2
        elif op == 0x4A:  # 'J' BININT
            stack.append(unpack_from("<i", data, i)[0])
            i += 4
        elif op == 0x8A:  # LONG1
            ln = data[i]
            stack.append(int.from_bytes(data[i + 1:i + 1 + ln], "little", signed=True))
            i += 1 + ln
        elif op == 0x86:  # TUPLE2
            b = stack.pop()
            a = stack.pop()
            stack.append((a, b))
        elif op == 0x85:  # TUPLE1
            stack.append((stack.pop(),))
        elif op == 0x87:  # TUPLE3
            c = stack.pop()
            b = stack.pop()
            a = stack.pop()
            stack.append((a, b, c))
        elif op == 0x74:  # 't' TUPLE
            k = len(stack) - 1 - stack[::-1].index(_MARK)
            items = tuple(stack[k + 1:])
            del stack[k:]
            stack.append(items)
        elif op == 0x29:  # ')' EMPTY_TUPLE
            stack.append(())
        elif op == 0x7D:  # '}' EMPTY_DICT
            stack.append({})
        elif op == 0x5D:  # ']' EMPTY_LIST
            stack.append([])
        elif op == 0x28:  # '(' MARK
            stack.append(_MARK)
        elif op == 0x75:  # 'u' SETITEMS
            k = len(stack) - 1 - stack[::-1].index(_MARK)
            d = stack[k - 1]
            if type(d) is not dict:
                raise RefusedOpcode("SETITEMS on non-dict")
            items = stack[k + 1:]
            for j in range(0, len(items), 2):
                d[items[j]] = items[j + 1]
            del stack[k:]
        elif op == 0x73:  # 's' SETITEM
            v = stack.pop()
            key = stack.pop()
            d = stack[-1]
            if type(d) is not dict:
                raise RefusedOpcode("SETITEM on non-dict")
            d[key] = v
        elif op == 0x65:  # 'e' APPENDS
            k = len(stack) - 1 - stack[::-1].index(_MARK)
            lst = stack[k - 1]
            if type(lst) is not list:
                raise RefusedOpcode("APPENDS on non-list")
            lst.extend(stack[k + 1:])
            del stack[k:]
        elif op == 0x61:  # 'a' APPEND
            v = stack.pop()
            lst = stack[-1]
            if type(lst) is not list:
                raise RefusedOpcode("APPEND on non-list")
            lst.append(v)
        elif op == 0x58:  # 'X' BINUNICODE
            ln = unpack_from("<I", data, i)[0]
            stack.append(data[i + 4:i + 4 + ln].decode("utf-8", "surrogatepass"))
            i += 4 + ln
        elif op == 0x8D:  # BINUNICODE8
            ln = unpack_from("<Q", data, i)[0]
            stack.append(data[i + 8:i + 8 + ln].decode("utf-8", "surrogatepass"))
            i += 8 + ln
        elif op == 0x71:  # 'q' BINPUT
            memo[data[i]] = stack[-1]
            i += 1
        elif op == 0x72:  # 'r' LONG_BINPUT
            memo[unpack_from("<I", data, i)[0]] = stack[-1]
            i += 4
        elif op == 0x47:  # 'G' BINFLOAT
            stack.append(unpack_from(">d", data, i)[0])
            i += 8
        elif op == 0x4E:  # 'N' NONE
            stack.append(None)
        elif op == 0x88:  # NEWTRUE
            stack.append(True)
        elif op == 0x89:  # NEWFALSE
            stack.append(False)
        elif op == 0x80:  # PROTO
            i += 1
        elif op == 0x95:  # FRAME
            i += 8
        elif op == 0x2E:  # '.' STOP
            if len(stack) != 1:
                raise RefusedOpcode("malformed pickle stack at STOP")
            return stack[0]
        else:
            raise RefusedOpcode(f"refusing pickle opcode 0x{op:02x} at byte {i - 1}: "
                                "only plain-data opcodes are interpreted")
    raise RefusedOpcode("pickle ended without STOP")


def load_snp_dict_pkl(path: str):
    """Load a reference SNP-dict cache (.pkl, .pkl.bz2 or .pkl.gz) without unpickling."""
    if path.endswith(".bz2"):
        with bz2.open(path, "rb") as fh:
            data = fh.read()
    elif path.endswith(".gz"):
        with gzip.open(path, "rb") as fh:
            data = fh.read()
    else:
        with open(path, "rb") as fh:
            data = fh.read()
    obj = safe_load_pickle_bytes(data)
    if not isinstance(obj, dict):
        raise ValueError("SNP cache does not hold a dict")
    return obj


def save_packed(path: str, packed) -> None:
    """Write a PackedSNPs (see sfs2d.pack) as a pickle-free .npz."""
    np.savez_compressed(
        path,
        counts=packed.counts,
        pos=packed.pos,
        chrom_off=packed.chrom_off,
        chrom_names=np.array(packed.chrom_names, dtype=np.str_),
        ann_id=packed.ann_id,
        ann_names=np.array(packed.ann_names, dtype=np.str_),
        pops=np.array([packed.pop1, packed.pop2], dtype=np.str_),
    )


def load_packed(path: str):
    from .pack import PackedSNPs

    z = np.load(path, allow_pickle=False)
    pops = [str(x) for x in z["pops"]]
    return PackedSNPs(
        counts=z["counts"],
        pos=z["pos"],
        chrom_off=z["chrom_off"],
        chrom_names=[str(x) for x in z["chrom_names"]],
        ann_id=z["ann_id"],
        ann_names=[str(x) for x in z["ann_names"]],
        pop1=pops[0],
        pop2=pops[1],
    )
