"""BUILD-CONTAINER ONLY: writes tests/golden/reference_line_counts.json, the number of lines
of every text file of the reference checkout (/root/reference) that citations may name.
Data only (path -> line count); tests/test_citations.py checks every `file.py:N` citation in
this repository against it, so a citation cannot point past the end of the file it names."""
import json
import os

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_line_counts.json")


def line_counts(ref=REF):
    counts = {}
    for root, dirs, files in os.walk(ref):
        dirs[:] = [d for d in dirs if d not in (".git", "__pycache__")]
        for fn in files:
            if fn.endswith((".py", ".yaml", ".md", ".sh", ".txt", ".cfg")):
                p = os.path.join(root, fn)
                with open(p, errors="ignore") as f:
                    counts[os.path.relpath(p, ref)] = sum(1 for _ in f)
    return counts


if __name__ == "__main__":
    c = line_counts()
    with open(OUT, "w") as f:
        json.dump(c, f, indent=0, sort_keys=True)
    print(len(c), "files ->", OUT)
