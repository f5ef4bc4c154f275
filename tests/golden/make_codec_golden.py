"""Regenerate tests/golden/codec_frames.json: the fixed-value frames of the reference's codec tests
(src/frame/serial/mod.rs:760-925, field values in oracle/codec.py reference_test_frames) encoded by
the Python codec oracle.  Run from the repo root: python tests/golden/make_codec_golden.py"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import codec as C  # noqa: E402


def main():
    rows = []
    for name, fr in C.reference_test_frames():
        fb = C.frame_write(fr)
        assert C.canonical(C.frame_read(fb)) == fr
        rows.append({"name": name, "len": len(fb), "hex": fb.hex()})
    with open(os.path.join(HERE, "codec_frames.json"), "w") as f:
        json.dump({"note": "frames of the reference's fixed-value codec tests (serial/mod.rs:760-925), encoded by "
                           "oracle/codec.py (restating serial/mod.rs:437-667 and build.rs)", "frames": rows}, f,
                  indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
