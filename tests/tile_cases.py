"""The tile kernel's layout grid (hysteria_amd/csrc/salamander_tile.h), shared by the
CPU-emulated tier (tests/test_emulated_kernels.py) and the GPU tier
(tests/test_gpu_parity.py::test_tile_layout_grid).

Slotted batches whose region edges are all multiples of 8.  Dense slots of 8 mod 16
(obfuscate 1200 -> 1208, deobfuscate 1216 -> 1208) and 0 mod 16, gapped slots (gap
bytes untouched), input strides with padding, partial last tiles, the 8-byte input
tail, 4096-byte input strides (64 KiB of staged LDS), slots needing several compose
passes (9000 B), every salt-word position of the PSK (lengths 4..127, including the
two-block case 121..127) and layouts that do not qualify (odd lengths, inputs over
4 KiB: the wave kernel).

("uniform", "n L obf"): in_stride = L (obfuscate) / L + 8 (deobfuscate of L + 8-byte
wire), dense output slots, PSK average_password.
("slotted", "n L obf slot_pad in_pad psk_len"): input stride L + in_pad, output slot
W + slot_pad with W = L + 8 (obfuscate) / L - 8 (deobfuscate), a PSK of psk_len bytes.
"""
TILE_CASES = [
    ("uniform", "257 1200 1"), ("uniform", "256 1200 0"), ("uniform", "301 1192 1"), ("uniform", "301 1192 0"),
    ("uniform", "33 16 1"), ("uniform", "33 24 0"), ("uniform", "300 17 1"), ("uniform", "99 1201 0"),
    ("slotted", "70 1200 1 24 8 16"), ("slotted", "70 1208 0 8 0 16"), ("slotted", "45 2040 1 0 16 9"),
    ("slotted", "37 4096 0 16 0 31"), ("slotted", "21 9000 1 0 0 16"), ("slotted", "40 64 1 0 0 4"),
    ("slotted", "40 64 0 0 24 5"), ("slotted", "23 100 1 4 4 16"), ("slotted", "30 1216 0 0 0 16"),
    ("slotted", "17 4096 1 8 0 16"), ("slotted", "17 4104 1 0 0 16"),
] + [("slotted", f"18 {L} 1 {pad} 0 {k}") for k, L, pad in
     [(4, 40, 0), (8, 48, 8), (12, 136, 0), (20, 200, 16), (60, 96, 0), (100, 1000, 8), (119, 512, 0),
      (120, 256, 0), (121, 256, 8), (124, 512, 0), (127, 264, 0), (128, 64, 0), (300, 1200, 0)]]




def slotted_params(which: str, args: str):
    """(n, L, obf, slot_pad, in_pad, psk) of a grid case, in the "slotted" form."""
    a = [int(x) for x in args.split()]
    if which == "uniform":
        n, L, obf = a
        if obf:
            return n, L, True, 0, 0, b"average_password"
        return n, L + 8, False, 0, 0, b"average_password"   # wire of L + 8 -> slots of L
    n, L, obf, slot_pad, in_pad, k = a
    return n, L, bool(obf), slot_pad, in_pad, bytes((7 * i + 1) & 0xFF for i in range(k))


def expects_tile(n, L, obf, slot_pad, in_pad):
    """tile_params (salamander_tile.h) for a 16-byte aligned input: does AUTO pick the tile kernel?"""
    W = L + 8 if obf else L - 8
    S, istride = W + slot_pad, L + in_pad
    return (L >= (16 if obf else 24) and L <= 4096 and istride <= 4096 and (L | S | istride) % 8 == 0
            and W <= S and S <= (1 << 20))
