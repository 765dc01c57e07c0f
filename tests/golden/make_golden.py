"""Writes tests/golden/appendix_b.json.

The reference ships no tests or fixtures and cannot be built in
this image (Boost.Heap is absent). The known answers below are the reference's
own behaviours as measured by the survey with the unmodified reference binary
(SURVEY.md Appendix B, §8a-R9/R10); each case cites the row it encodes. The
expected distance vectors are written out from those recorded observations by
hand — nothing here is computed by this repository's code.

Run: python tests/golden/make_golden.py   (deterministic; output committed)
"""
import hashlib
import json
import os

INF = "inf"


def sol(values):
    """sol_file bytes for a list of ints / 'inf' (output_vector :32-46)."""
    return "the vector is:\n" + "".join(f"{v}\n" for v in values)


CASES = [
    # name, text, argv source string, expected distances or error, Appendix B row
    ("crlf", "0\t1\r\n1\t2\r\n", "0", [0, 1, 2], "CRLF lines: CR is whitespace to >>"),
    ("leading_space", " 0\t1\n0 2\n", "0", [0, INF, 1],
     "leading space -> line skipped; space-separated '0 2' accepted"),
    ("comments_blank", "# Directed graph\n\n0\t1\n# mid comment\n\n1\t2\n", "0", [0, 1, 2],
     "blank lines and # comments anywhere are skipped"),
    ("signed_first_byte", "0 1\n+3 4\n-1 2\n", "0", [0, 1], "'+3 4', '-1 2' skipped (byte 0 not a digit)"),
    ("three_columns", "0 1 5\n1 2 7\n", "0", [0, 1, 2], "3rd column ignored -> unit weight"),
    ("dups_selfloops", "0 0\n0 1\n0 1\n1 1\n1 0\n", "0", [0, 1], "duplicate edges and self-loops kept, no effect"),
    ("bad_second_field", "0 1\n2 x\n", "2", [1, 2, 0], "'2 x' -> dest parsed as 0 -> edge 2->0"),
    ("absent_ids", "0 3\n", "0", [0, INF, INF, 1], "ids absent from file but < max appear as inf (N = max+1)"),
    ("source_ge_n", "0 1\n1 2\n", "9", [INF, INF, INF], "source 9 (>= N) -> all inf"),
    ("source_negative", "0 1\n1 2\n", "-1", [INF, INF, INF], "source -1 -> all inf"),
    ("source_atoi_alpha", "0 1\n1 2\n", "abc", [0, 1, 2], "atoi('abc') = 0"),
    ("source_atoi_suffix", "0 1\n1 2\n2 0\n", "2x", [1, 2, 0], "atoi('2x') = 2"),
    ("source_atoi_space", "0 1\n1 2\n2 0\n", " 1", [2, 0, 1], "atoi(' 1') = 1"),
    ("empty_file", "", "0", [], "N = 0 -> header only"),
    ("single_field", "0 1\n5\n", "0", "parse_error",
     "single-field line: dest uninitialised (UB) -> the build rejects it; not a parity target"),
]


def main():
    out = []
    for name, text, src, exp, row in CASES:
        case = {"name": name, "text": text, "source": src, "appendix_b": row}
        if exp == "parse_error":
            case["expect"] = "parse_error"
        else:
            case["expect"] = [100000 if v == INF else v for v in exp]
            case["sol"] = sol(exp)
        out.append(case)
    # chain of 100,010 vertices (Appendix B: ids >= 100,000 print inf)
    n = 100010
    chain_sol = sol([i if i < 100000 else INF for i in range(n)])
    out.append({"name": "chain_100010", "generator": "chain", "n": n, "source": "0",
                "appendix_b": "chain of 100,010: node 99,999 -> 99999, node 100,000 -> inf",
                "sol_sha256": hashlib.sha256(chain_sol.encode()).hexdigest(),
                "sol_bytes": len(chain_sol)})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "appendix_b.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(f"wrote {path}: {len(out)} cases")


if __name__ == "__main__":
    main()
