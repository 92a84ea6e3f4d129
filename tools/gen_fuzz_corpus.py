#!/usr/bin/env python3
"""Seed corpus of csrc/tests/fuzz_deflate_tmpl.cc (tests/fuzz_corpus/deflate_tmpl/): one input
per layout the fuzzer must reach on purpose -- a label over the 32 KB window, blank runs over
258 bytes, empty and one-byte segments, every byte value in static text, code rebuilds between
patches -- in the input grammar the target reads (first byte = segment count - 1, ...)."""
import os
import random

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "fuzz_corpus", "deflate_tmpl")


def seg_generic(fields, static=b"\x05abcde", tail=b"\x02}\n"):
    """kind 2 segment: nf fields, each a static chunk then a field (width byte, wide flag, value)."""
    b = bytes([2, len(fields)])
    for width_code, wide, value in fields:
        b += static + bytes([width_code, 0 if wide else 1])
        if wide:
            b += bytes([wide])
        b += bytes([len(value) - 1]) + value
    return b + tail


def main() -> None:
    os.makedirs(OUT, exist_ok=True)
    rng = random.Random(6)
    seeds = {
        # 3 segments of 2 fields, parsed as one run, 3 patch rounds with a rebuild
        "basic": bytes([2]) + seg_generic([(9, 0, b"42"), (23, 0, b"3.5e+10")]) * 3
        + bytes([0, 3]) + b"\x00\x01" * 6 + b"\x00",
        # a label longer than 32 KB (static code 255: 32768 + n repeats), then a field behind it
        "long_label": bytes([0, 2, 1, 255, 0x10, 0x00, ord("q"), 5, 1, 2]) + b"777" + b"\x00" + bytes([0, 2]) + b"\x00" * 8,
        # blank runs over 258 bytes: width = 259 + byte when the flag byte % 16 == 0
        "long_pad": bytes([0, 2, 2]) + b"\x03abc" + bytes([9, 0, 200, 0]) + b"1" + b"\x03def" + bytes([9, 0, 255, 1]) + b"22"
        + b"\x00" + bytes([1, 4]) + b"\x00\x01" * 8,
        # empty, one-byte, empty, one-byte segments; each parsed on its own (provisional)
        "tiny_segments": bytes([3, 0, 1, ord("#"), 0, 1, 0xff, 1, 2]),
        # every byte value in static text (static code 254), fields around it
        "all_bytes": bytes([1]) + bytes([2, 2, 254, 5, 1, 0]) + b"9" + bytes([254, 7, 1, 3]) + b"-1e9" + b"\x00"
        + bytes([2, 1, 3]) + b"\x00\x02" * 12,
        # code rebuilds between every patch round (rebuild byte % 4 == 0)
        "rebuilds": bytes([1]) + seg_generic([(30, 0, b"123456789"), (3, 0, b"7")]) * 2 + bytes([2, 7])
        + (b"\x00" * 4 + b"\x00") * 7,
    }
    for k in range(10):  # random bodies for breadth
        seeds[f"random_{k}"] = bytes(rng.randrange(256) for _ in range(rng.randrange(64, 2048)))
    for name, data in seeds.items():
        with open(os.path.join(OUT, name), "wb") as fh:
            fh.write(data)
    print(f"{len(seeds)} seeds in {OUT}")


if __name__ == "__main__":
    main()
