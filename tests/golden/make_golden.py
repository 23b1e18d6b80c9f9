"""Generate the committed golden fixtures under tests/golden/.

Run once in the build container (it reads the reference checkout as DATA only):

    python tests/golden/make_golden.py /root/reference

Fixtures and where their expected values come from:

* ``host_known_answer.npz`` -- the reference's only known-answer test:
  ``repository/src/host.c:7`` (4096 elements), ``:20-25`` (``in[i] = i*(rank+1)``),
  ``:51-55`` (``dst[i] == 3*i`` for two ranks).  The generator reads those
  constants from host.c and asserts the pattern is unchanged.
* ``icrc_test_c.json`` -- the canned RoCEv2 ACK frame of
  ``repository/src/test.c:4-20`` with the ICRC bytes kept in the comment at
  ``test.c:21`` (``0xe8, 0xb0, 0xbb, 0x30``), captured from a real soft-RoCE
  stack; the frame also carries the IPv4 header checksum that stack wrote.
* ``sum_edge.npz`` -- int32 lanes at the wrap edges (INT32_MIN/MAX, -1, 0, ...)
  for 2..8 ranks; expected sums by exact Python integer arithmetic mod 2^32 (the
  switch semantics of ``non_termination_switch.c:361-363``).
* ``quant_kat.json`` -- fp32 -> fixed-point known answers derived from the spec
  with exact rational arithmetic (``fractions.Fraction``, round-half-even), not
  from the C oracle: powers of two, ties, saturation, NaN/Inf, subnormals.
"""
from __future__ import annotations

import json
import math
import os
import re
import struct
import sys
from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
INT32_MIN, INT32_MAX = -(2 ** 31), 2 ** 31 - 1


def f32_bits(x: float) -> int:
    return struct.unpack("<I", struct.pack("<f", x))[0]


def bits_f32(b: int) -> float:
    return struct.unpack("<f", struct.pack("<I", b))[0]


def quant_exact(bits: int, k: int) -> int:
    x = bits_f32(bits)
    if math.isnan(x):
        return 0
    if math.isinf(x):
        return INT32_MAX if x > 0 else INT32_MIN
    v = Fraction(x) * (Fraction(2) ** k)
    q = round(v)                      # Fraction.__round__: half to even
    return max(INT32_MIN, min(INT32_MAX, q))


def host_known_answer(ref: str) -> None:
    src = open(os.path.join(ref, "repository/src/host.c")).read()
    m = re.search(r"#define\s+IN_DATA_COUNT\s+(\d+)", src)
    assert m, "host.c: IN_DATA_COUNT not found"
    count = int(m.group(1))
    assert "in_data[i] = i * (rank+1);" in src, "host.c input pattern changed"
    assert "assert(dst_data[i] == 3 * i);" in src, "host.c expected pattern changed"
    inputs = np.stack([np.arange(count, dtype=np.int64) * (r + 1) for r in range(2)]).astype(np.int32)
    expected = (np.arange(count, dtype=np.int64) * 3).astype(np.int32)
    np.savez(os.path.join(HERE, "host_known_answer.npz"), inputs=inputs, expected=expected,
             comm_size_bytes=np.int64(count * 4))


def icrc_test_c(ref: str) -> None:
    src = open(os.path.join(ref, "repository/src/test.c")).read()
    body = src[src.index("uint8_t pack[1024] = {"):src.index("};")]
    lines = body.split("\n")
    frame, kept = [], None
    for ln in lines[1:]:
        s = ln.strip()
        if s.startswith("//"):
            kept = [int(t, 16) for t in re.findall(r"0x([0-9a-fA-F]{2})", s)]
            continue
        code = s.split("//")[0]
        frame += [int(t, 16) for t in re.findall(r"0x([0-9a-fA-F]{2})", code)]
    assert len(frame) == 58 and kept is not None and len(kept) == 4, (len(frame), kept)
    icrc_le = int.from_bytes(bytes(kept), "little")   # test.c:32-33 stores the CRC host-order (LE)
    ip_csum = (frame[24] << 8) | frame[25]
    json.dump({
        "source": "repository/src/test.c:4-22",
        "frame_hex": bytes(frame).hex(),
        "icrc_bytes_hex": bytes(kept).hex(),
        "icrc_u32": icrc_le,
        "ipv4_checksum": ip_csum,
    }, open(os.path.join(HERE, "icrc_test_c.json"), "w"), indent=1)


def sum_edge() -> None:
    edge = [INT32_MIN, INT32_MAX, -1, 0, 1, INT32_MIN + 1, INT32_MAX - 1, 0x40000000, -0x40000000, 12345]
    rng = np.random.default_rng(20251015)
    out = {}
    for R in range(2, 9):
        n = 1024 + 37   # ragged: not a multiple of the 4-lane vector
        x = rng.integers(INT32_MIN, INT32_MAX, size=(R, n), dtype=np.int64, endpoint=True)
        for j, v in enumerate(edge):   # edge lanes in every rank, rotated
            for r in range(R):
                x[r, (j * 7 + r) % n] = edge[(j + r) % len(edge)]
        x[:, :4] = INT32_MAX            # all ranks max -> wraps
        x[:, 4:8] = INT32_MIN
        s = x.sum(axis=0)
        s = ((s + 2 ** 31) % 2 ** 32) - 2 ** 31
        out[f"in_R{R}"] = x.astype(np.int32)
        out[f"sum_R{R}"] = s.astype(np.int32)
    np.savez(os.path.join(HERE, "sum_edge.npz"), **out)


def quant_kat() -> None:
    xs = [0.0, -0.0, 1.0, -1.0, 0.5, 1.5, 2.5, -2.5, 3.5, 1e-3, -7.25, 6.0, 123.456,
          float("inf"), float("-inf"), float("nan"), 3.4028234663852886e38, -3.4028234663852886e38,
          1.401298464324817e-45, -1.401298464324817e-45, 1.1754943508222875e-38, 64.0, -64.0, 63.99999618530273]
    ks = [0, 1, 8, 23, 25, 30, 31, -1, -8, 64, -64]
    cases = []
    for k in ks:
        for x in xs:
            b = f32_bits(x) if not math.isnan(x) else 0x7FC00000
            cases.append({"bits": b, "k": k, "q": quant_exact(b, k)})
    # exact ties at every k in a range: (m + 0.5) * 2^-k
    for k in range(0, 26, 5):
        for m in (-3, -2, -1, 0, 1, 2, 3, 1000, 1001):
            x = (m + 0.5) * 2.0 ** -k
            b = f32_bits(x)
            cases.append({"bits": b, "k": k, "q": quant_exact(b, k)})
    # saturation boundaries at k = 0: the largest float below 2^31, 2^31, -2^31, just past it
    for x in (2147483520.0, 2147483648.0, -2147483648.0, -2147483904.0):
        b = f32_bits(x)
        cases.append({"bits": b, "k": 0, "q": quant_exact(b, 0)})
    json.dump({"spec": "q = sat_int32(round_half_even(x * 2^k)); NaN -> 0", "cases": cases},
              open(os.path.join(HERE, "quant_kat.json"), "w"))


def nonroot_down_survey() -> None:
    """The one recorded output of the reference's non-root branches (SURVEY.md
    section 0, line 28, from driving its pipeline() as a non-root): a child
    decoded 234881024 where the parent sent 14 -- 0x0000000E with its bytes
    reversed (nts.c:413 keeps the wire bytes, util.c:403-405 htonls them again)."""
    parent = 14
    child = int.from_bytes(parent.to_bytes(4, "big"), "little")
    assert child == 234881024
    json.dump({"source": "SURVEY.md section 0 (line 28): the reference's own pipeline() driven as a non-root "
                         "switch (nts.c:408-419) -- a child received 234881024 for a parent value of 14",
               "parent_value": parent, "child_value": child,
               "note": "the child's value is what a host decodes with ntohl (api.c:428-430) from the word the "
                       "non-root sent down"},
              open(os.path.join(HERE, "nonroot_down_survey.json"), "w"), indent=1)


def main() -> None:
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    host_known_answer(ref)
    icrc_test_c(ref)
    sum_edge()
    quant_kat()
    nonroot_down_survey()
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
