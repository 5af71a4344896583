"""sha256 over the HIP library's sources (csrc/*.hip, csrc/*.h, include/*.h, file names
included). Torch-free, so the Makefile can run it as a script and compile the value into the
library (ob_source_digest); _lib.load() refuses a library whose digest differs from the
sources next to it (a stale build)."""
from __future__ import annotations

import hashlib
from pathlib import Path

PKG = Path(__file__).resolve().parents[1]


def source_digest(pkg: Path = PKG) -> str:
    files = sorted(list((pkg / "csrc").glob("*.hip")) + list((pkg / "csrc").glob("*.h")) +
                   list((pkg.parent / "include").glob("*.h")))
    h = hashlib.sha256()
    for f in files:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()


if __name__ == "__main__":
    print(source_digest())
