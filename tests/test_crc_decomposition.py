"""CPU check of the CRC kernel's decomposition (no GPU): a Python emulation of exactly the
chunking, position-based init injection, two fold chains per lane, per-lane zero advance to the
window end, 16-lane XOR reduce and window chaining that crc32c.hip (crc_frames_kernel: 16 lanes x
64 bytes per 1 KiB window) performs, compared with the oracle.  A wrong index formula shows up
here before it costs a GPU run."""
import random

Q, S = 16, 64


def _raw(orc, reg, data):
    """CRC register after absorbing `data` from `reg` (no final inversion)."""
    return orc.crc32c_update(reg, bytes(data))


def _zero_advance(orc, reg, nbytes):
    return _raw(orc, reg, bytes(nbytes))


def emulate(orc, buf, o, L, init, Q, S):
    W = Q * S
    E = o + L
    nw = (L + W - 1) // W
    R = 0
    for wi in range(nw):
        acc = 0
        for gl in range(Q):
            be = E - (nw - 1 - wi) * W - (Q - 1 - gl) * S
            cs = be - S
            bs = max(cs, o)
            cnt = max(be - bs, 0)
            p0 = bs - o
            data = bytearray(buf[bs:bs + cnt])
            for i in range(cnt):
                if p0 + i < 4:
                    data[i] ^= (init >> (8 * (p0 + i))) & 0xFF
            # the lane's 64-byte chunk (zero bytes before the frame start): two chains of 32
            # bytes joined by a 32-zero-byte advance, then advanced over 64 (15 - gl) zero bytes
            chunk = bytes(S - cnt) + bytes(data)
            r = _zero_advance(orc, _raw(orc, 0, chunk[:S // 2]), S // 2) ^ _raw(orc, 0, chunk[S // 2:])
            acc ^= _zero_advance(orc, r, S * (Q - 1 - gl)) if cnt else 0
        regs = [acc]
        R = _zero_advance(orc, R, W) ^ regs[0]
    state = R ^ ((init >> (8 * L)) if L < 4 else 0)
    return (~state) & 0xFFFFFFFF


def test_decomposition_matches_oracle(orc):
    rng = random.Random(Q * 1000 + S)
    buf = bytes(rng.getrandbits(8) for _ in range(3 * Q * S + 64))
    lengths = [0, 1, 2, 3, 4, 5, 7, 8, 63, 64, 65, S - 1, S, S + 1, S + 2, S + 3, Q * S - 1, Q * S, Q * S + 1,
               Q * S + 2, Q * S + 3, 2 * Q * S + 5]
    for L in lengths:
        for o in (0, 1, 3, 8):
            for init in (0xFFFFFFFF, 0x12345678):
                want = (~orc.crc32c_update(init, buf[o:o + L])) & 0xFFFFFFFF
                assert emulate(orc, buf, o, L, init, Q, S) == want, (Q, S, L, o, hex(init))
