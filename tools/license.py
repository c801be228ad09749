"""SPDX header check / fix for native sources (reference: hack/boilerplate + license tooling).

    python tools/license.py          # list files without an SPDX line (exit 1 if any)
    python tools/license.py --fix    # prepend `// SPDX-License-Identifier: Apache-2.0`
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPDX = "SPDX-License-Identifier: Apache-2.0"
EXTS = {".cpp": "//", ".h": "//", ".hip": "//", ".cc": "//"}
DIRS = ("csrc",)


def files():
    for d in DIRS:
        for dp, _, fs in os.walk(os.path.join(ROOT, d)):
            for f in sorted(fs):
                ext = os.path.splitext(f)[1]
                if ext in EXTS:
                    yield os.path.join(dp, f), EXTS[ext]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--fix", action="store_true")
    a = ap.parse_args(argv)
    missing = []
    for path, cmt in files():
        with open(path) as f:
            text = f.read()
        if SPDX in "\n".join(text.splitlines()[:3]):
            continue
        missing.append(os.path.relpath(path, ROOT))
        if a.fix:
            with open(path, "w") as f:
                f.write(f"{cmt} {SPDX}\n" + text)
    if missing and not a.fix:
        print("missing SPDX header:\n  " + "\n  ".join(missing))
        return 1
    print(f"{'fixed' if a.fix else 'ok'}: {len(missing)} file(s) {'updated' if a.fix else 'missing'}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
