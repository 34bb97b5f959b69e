#!/usr/bin/env python3
"""Extract the reference codec's constant tables into a binary blob.

TEST/BUILD INFRASTRUCTURE.  The MELPe codebooks and filter tables are data of
the standard (e.g. melpe/qnt12_cb.c, melpe/fsvq_cb.c, melpe/coeff.c,
melpe/math_lib.c:33 log_table).  Bit-exact parity needs the exact values, so
instead of transcribing them this script reads them out of the reference's
compiled object files (oracle/_ref/obj/*.o, built from the sources where they
lie by oracle/Makefile) with a minimal ELF64 reader, and writes

  pairphone_amd/data/melpe_tables.bin   little-endian int16 words
  pairphone_amd/csrc/tables_gen.h       name -> (word offset, count) only

Both are committed so the GPU box (which has no /root/reference) can build.
Function-local statics (e.g. the sin/cos/pow10 tables in math_lib.c) have
compiler-numbered names; they are identified by size and first value.
"""
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OBJ = os.path.join(HERE, "_ref", "obj")
ROOT = os.path.dirname(HERE)

# (our name, object file, symbol name or (prefix, nwords, first_value), words)
TABLES = [
    ("enhpf_coef", "classify", "enhpf_coef", 17),
    ("enlpf_coef", "classify", "enlpf_coef", 17),
    ("bpf_den_class", "coeff", "bpf_den_class", 7),
    ("bpf_num_class", "coeff", "bpf_num_class", 7),
    ("lpf_den", "coeff", "lpf_den", 9),
    ("lpf_num", "coeff", "lpf_num", 9),
    ("bpf_den", "coeff", "bpf_den", 45),
    ("bpf_num", "coeff", "bpf_num", 45),
    ("disp_cof", "coeff", "disp_cof", 65),
    ("bp_cof", "coeff", "bp_cof", 165),
    ("win_cof", "coeff", "win_cof", 200),
    ("syntab74", "fec_code", "syntab74", 8),
    ("pmat74", "fec_code", "pmat74", 12),
    ("pmat84", "fec_code", "pmat84", 16),
    ("syntab84", "fec_code", "syntab84", 16),
    ("pitch_enc", "fec_code", "pitch_enc", 100),
    ("pitch_dec", "fec_code", "pitch_dec", 128),
    ("low_rate_pitch_enc", "fec_code", "low_rate_pitch_enc", 396),
    ("low_rate_pitch_dec", "fec_code", "low_rate_pitch_dec", 512),
    ("fsvq_cb", "fsvq_cb", "fsvq_cb", 2560),
    ("lagw_cof", "lpc_lib", ("lagw_cof.", 16, None), 16),
    ("pow10_q_table", "math_lib", ("Q_table.", 4, None), 4),
    ("pow10_tens_table", "math_lib", ("tens_table.", 9, None), 9),
    ("sin_table", "math_lib", ("table.", 129, 0), 129),
    ("cos_table", "math_lib", ("table.", 129, 32767), 129),
    ("log_table", "math_lib", "log_table", 256),
    ("pow10_table", "math_lib", ("table.", 257, 2048), 257),
    ("bit_order", "melp_chn", "bit_order", 81),
    ("dc_den", "melp_sub", ("dc_den.", 9, None), 9),
    ("dc_num", "melp_sub", ("dc_num.", 9, None), 9),
    ("wtr_front", "npp", ("wtr_front.", 32, None), 32),
    ("sqrt_tukey_256_180", "npp", "sqrt_tukey_256_180", 256),
    ("lpar", "pitch", ("lpar.", 4, None), 4),
    ("hpf60_den", "postfilt", ("hpf60_den.", 3, None), 3),
    ("hpf60_num", "postfilt", ("hpf60_num.", 3, None), 3),
    ("lpf3500_den", "postfilt", ("lpf3500_den.", 3, None), 3),
    ("lpf3500_num", "postfilt", ("lpf3500_num.", 3, None), 3),
    ("syn_inp", "postfilt", ("syn_inp.", 4, None), 4),
    ("inv_bp_index_map", "qnt12_cb", "inv_bp_index_map", 4),
    ("vvv_index_map", "qnt12_cb", "vvv_index_map", 4),
    ("pitch_uvflag_map", "qnt12_cb", "pitch_uvflag_map", 9),
    ("bp_index_map", "qnt12_cb", "bp_index_map", 16),
    ("inpCoef", "qnt12_cb", "inpCoef", 320),
    ("pitch_vq_cb_uvv", "qnt12_cb", "pitch_vq_cb_uvv", 1536),
    ("lsp_v_256x64x32x32", "qnt12_cb", "lsp_v_256x64x32x32", 3840),
    ("lsp_uv_9", "qnt12_cb", "lsp_uv_9", 5120),
    ("gain_vq_cb", "qnt12_cb", "gain_vq_cb", 6144),
    ("pitch_vq_cb_vvv", "qnt12_cb", "pitch_vq_cb_vvv", 6144),
    ("res256x64x64x64", "qnt12_cb", "res256x64x64x64", 8960),
    # 2400 bps MELP (melpe/msvq_cb.c:37,41): the 4-stage LSF MSVQ, Q17, and
    # its mean vector, Q15 (appended: earlier offsets are unchanged)
    ("msvq_cb_mean", "msvq_cb", "msvq_cb_mean", 10),
    ("msvq_cb", "msvq_cb", "msvq_cb", 3200),
]


def read_elf_symbols(path):
    data = open(path, "rb").read()
    assert data[:4] == b"\x7fELF" and data[4] == 2 and data[5] == 1, path
    e_shoff, = struct.unpack_from("<Q", data, 0x28)
    e_shentsize, e_shnum, e_shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = []
    for i in range(e_shnum):
        off = e_shoff + i * e_shentsize
        name, typ, flags, addr, offset, size, link, info, align, entsize = \
            struct.unpack_from("<IIQQQQIIQQ", data, off)
        secs.append(dict(name=name, type=typ, offset=offset, size=size,
                         link=link, entsize=entsize))
    shstr = secs[e_shstrndx]

    def cstr(sec, idx):
        start = sec["offset"] + idx
        end = data.index(b"\0", start)
        return data[start:end].decode()

    for s in secs:
        s["sname"] = cstr(shstr, s["name"])
    syms = {}
    for s in secs:
        if s["type"] != 2:  # SHT_SYMTAB
            continue
        strtab = secs[s["link"]]
        for j in range(s["size"] // 24):
            st_name, st_info, st_other, st_shndx, st_value, st_size = \
                struct.unpack_from("<IBBHQQ", data, s["offset"] + j * 24)
            if st_shndx == 0 or st_shndx >= len(secs) or st_size == 0:
                continue
            sec = secs[st_shndx]
            if sec["type"] == 8:  # NOBITS
                continue
            nm = cstr(strtab, st_name)
            raw = data[sec["offset"] + st_value: sec["offset"] + st_value + st_size]
            syms.setdefault(nm, raw)
    return syms


def main():
    blob = bytearray()
    manifest = []
    cache = {}
    for ours, obj, sym, words in TABLES:
        if obj not in cache:
            cache[obj] = read_elf_symbols(os.path.join(OBJ, obj + ".o"))
        syms = cache[obj]
        if isinstance(sym, tuple):
            prefix, n, first = sym
            cands = [k for k, v in syms.items()
                     if k.startswith(prefix) and len(v) == 2 * n and
                     (first is None or struct.unpack_from("<h", v, 0)[0] == first)]
            assert len(cands) == 1, (ours, cands)
            raw = syms[cands[0]]
        else:
            raw = syms[sym]
        assert len(raw) == 2 * words, (ours, len(raw), words)
        manifest.append((ours, len(blob) // 2, words))
        blob += raw
    os.makedirs(os.path.join(ROOT, "pairphone_amd", "data"), exist_ok=True)
    with open(os.path.join(ROOT, "pairphone_amd", "data", "melpe_tables.bin"), "wb") as f:
        f.write(blob)
    lines = [
        "/* GENERATED by oracle/dump_tables.py -- do not edit.",
        " * Word offsets/counts of the constant tables inside",
        " * pairphone_amd/data/melpe_tables.bin (int16, little endian). */",
        "#ifndef MELPE_TABLES_GEN_H",
        "#define MELPE_TABLES_GEN_H",
        "#define MELPE_TABLE_WORDS %d" % (len(blob) // 2),
    ]
    for ours, off, words in manifest:
        lines.append("#define TOFF_%s %d" % (ours, off))
        lines.append("#define TLEN_%s %d" % (ours, words))
    lines.append("#endif")
    with open(os.path.join(ROOT, "pairphone_amd", "csrc", "tables_gen.h"), "w") as f:
        f.write("\n".join(lines) + "\n")
    json.dump(manifest, open(os.path.join(HERE, "_ref", "tables_manifest.json"), "w"))
    print("wrote %d words in %d tables" % (len(blob) // 2, len(manifest)))


if __name__ == "__main__":
    sys.exit(main())
