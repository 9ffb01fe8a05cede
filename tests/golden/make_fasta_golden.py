#!/usr/bin/env python3
"""Generates tests/golden/fasta_cases.json: crafted FASTA/FASTQ files and the first
record the REFERENCE's reader returns for each (sequence_io.cpp, compiled by
`make -C oracle ref` into oracle/_ref/ref_fasta; needs /root/reference, so this
runs in the build container only -- the JSON is the committed fixture).

Usage: python tests/golden/make_fasta_golden.py
"""
import json
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

CASES = [
    ("simple.fa", b">chr1 test\nACGT\nTTGA\n>chr2\nGGGG\n"),
    ("no_final_newline.fna", b">x\nACGTACGT\nAC"),
    ("crlf.fasta", b">crlf\r\nACGT\r\nAACC\r\n"),
    ("lower_n.fa", b">m\nacgtNNNNacgt\nRYKM\n\n>n\nA\n"),
    ("blank_lines.fa", b">b\n\nAC\n\nGT\n"),
    ("single_record.fa", b">only\n" + b"ACGT" * 40 + b"\n"),
    ("empty_seq.fa", b">e\n>f\nACGT\n"),
    ("no_header.fa", b"ACGT\n"),
    ("reads.fq", b"@r1\nACGTTGCA\n+\nIIIIIIII\n@r2\nGG\n+\nII\n"),
    ("sniff_fasta.txt", b">s\nCCGG\nAA\n"),
    ("sniff_fastq.seq", b"@q\nTTAA\n+\n!!!!\n"),
    ("unknown.txt", b"hello\n"),
]


def main():
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_fasta")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"])
    out = []
    with tempfile.TemporaryDirectory() as td:
        for name, data in CASES:
            path = os.path.join(td, name)
            with open(path, "wb") as f:
                f.write(data)
            line = subprocess.run([exe, path], capture_output=True, text=True, check=True).stdout.strip()
            parts = line.split(" ", 1)
            if parts[0] == "ok":
                h, d, _ = parts[1].split(" ")
                res = {"ok": True, "header": h, "data": d}
            else:
                res = {"ok": False, "error": line}
            out.append({"name": name, "content": data.hex(), **res})
    with open(os.path.join(HERE, "fasta_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_fasta_golden.py (reference sequence_io.cpp)", "cases": out},
                  f, indent=1)
    print(f"{len(out)} cases")


if __name__ == "__main__":
    main()
