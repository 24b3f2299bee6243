"""LDS slot conflicts of the four-step spectral kernel's bin exchange (dev tool, CPU): for N = 2048 / 1024 / 512,
the worst number of lanes of a half wave on one 8-byte slot (32 slots of 64 banks), for the own-bin writes and the
mirror-bin reads, under candidate paddings of the natural bin index (vqa_spectral.hip Spec4::slot uses the last).
    python tools/spec4_banks.py
"""
import itertools
def bitrev(x, bits):
    return int(format(x, f'0{bits}b')[::-1], 2) if bits else 0
def layout(N, h_of_g):
    P = N // 64; G = 64 // P
    own = {}  # (lane, q) -> k
    for L in range(64):
        k1, g = divmod(L, G)
        for q in range(P):
            own[(L, q)] = k1 + P * (q + P * h_of_g(g, G))
    return own
def worst(addrs):
    # addrs: per lane complex index (8B); half-waves of 32 lanes; 64 banks x 4B -> 32 slots of 8B
    w = 0
    for half in (range(32), range(32, 64)):
        slots = {}
        for L in half:
            s = addrs[L] % 32
            slots[s] = slots.get(s, 0) + 1
        w = max(w, max(slots.values()))
    return w
for N in (2048, 1024, 512):
    P = N // 64; G = 64 // P
    bits = G.bit_length() - 1
    own = layout(N, lambda g, G: bitrev(g, bits))
    for name, pad in [("none", lambda k: k), ("k>>5", lambda k: k + (k >> 5)), ("k>>4", lambda k: k + (k >> 4)),
                      ("k>>3", lambda k: k + (k >> 3)), ("k/P", lambda k: k + k // P),
                      ("k/(P*P)*?", lambda k: k + (k // (P * P)) * (32 // G))]:
        ww = wr = 0
        for q in range(P):
            ww = max(ww, worst([pad(own[(L, q)]) for L in range(64)]))
            wr = max(wr, worst([pad((N - own[(L, q)]) % N) for L in range(64)]))
        print(N, name, "write", ww, "read", wr)
