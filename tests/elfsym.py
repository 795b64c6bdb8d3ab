"""A minimal ELF64 symbol lookup (no pyelftools here): the file offset and
value of a global data symbol in a code object, for the workspace-size
checks in tests/test_gen_meta.py."""
import struct


def symbol_offset(path, name):
    """(file offset, size) of symbol `name` in the ELF64 file at `path`"""
    with open(path, "rb") as f:
        data = f.read()
    assert data[:4] == b"\x7fELF" and data[4] == 2, "not ELF64"
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + k * shentsize) for k in range(shnum)]
    for sec in secs:
        if sec[1] != 2:          # SHT_SYMTAB
            continue
        strtab = secs[sec[6]]
        for k in range(sec[5] // 24):
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from(
                "<IBBHQQ", data, sec[4] + 24 * k)
            s0 = strtab[4] + st_name
            nm = data[s0:data.index(b"\0", s0)].decode()
            if nm == name:
                tgt = secs[st_shndx]
                return tgt[4] + (st_value - tgt[3]), st_size
    raise KeyError(name)


def read_u32(path, name):
    off, size = symbol_offset(path, name)
    assert size == 4
    with open(path, "rb") as f:
        f.seek(off)
        return struct.unpack("<I", f.read(4))[0]
