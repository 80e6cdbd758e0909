#!/usr/bin/env python3
"""Extract the file-level expectations of the reference's TestMatch suite
(tools/test/TestMatch.cc:154-355 OrcFileDescription table, :1029+
makeMetadata) into tests/golden/testmatch.json: per example file its
expected-output JSON name, type string, format version, software version,
row count, content length, stripe count, compression, compression block
size, row index stride and user metadata (hex). Run in the container where
/root/reference exists; the JSON is the committed fixture (data only)."""
import json
import os
import re
import sys

SRC = "/root/reference/tools/test/TestMatch.cc"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "testmatch.json")


def c_strings(tok):
    """Concatenated C string literals -> str (with \\x escapes)."""
    parts = re.findall(r'"((?:[^"\\]|\\.)*)"', tok)
    s = "".join(parts)
    return bytes(s, "latin-1").decode("unicode_escape")


def split_args(body):
    out, depth, cur, in_str, esc = [], 0, "", False, False
    for ch in body:
        if in_str:
            cur += ch
            if esc:
                esc = False
            elif ch == "\\":
                esc = True
            elif ch == '"':
                in_str = False
            continue
        if ch == '"':
            in_str = True
            cur += ch
        elif ch in "([<":
            depth += 1
            cur += ch
        elif ch in ")]>":
            depth -= 1
            cur += ch
        elif ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def main():
    src = open(SRC).read()
    meta = {}
    m = re.search(r"makeMetadata\(\) \{(.*?)return result;", src, re.S)
    body = m.group(1)
    for k, v in re.findall(r'result\["([^"]+)"\] = ((?:"(?:[^"\\]|\\.)*"\s*)+);', body):
        meta[k] = c_strings(v).encode("latin-1").hex()
    buf = re.search(r"buffer\[\] = \{(.*?)\};", body, re.S).group(1)
    bigkey = re.search(r'result\["([^"]+)"\] = std::string\(', body)
    if bigkey:
        meta[bigkey.group(1)] = bytes(int(x) for x in re.findall(r"\d+", buf)).hex()
    rows = []
    for m in re.finditer(r"OrcFileDescription\(", src):
        i = m.end()
        depth, j = 1, i
        while depth:
            if src[j] == "(":
                depth += 1
            elif src[j] == ")":
                depth -= 1
            j += 1
        args = split_args(src[i:j - 1])
        if len(args) != 12 or not args[0].startswith('"'):
            continue
        rows.append({
            "file": c_strings(args[0]), "json": c_strings(args[1]), "type": c_strings(args[2]),
            "format_version": c_strings(args[3]), "software_version": c_strings(args[4]),
            "rows": int(args[5].rstrip("UL")), "content_length": int(args[6]), "stripes": int(args[7]),
            "compression": args[8].replace("CompressionKind_", ""), "compression_size": int(args[9]),
            "row_index_stride": int(args[10]),
            "metadata": meta if "makeMetadata" in args[11] else {},
        })
    json.dump(rows, open(OUT, "w"), indent=1)
    print("%d descriptions -> %s" % (len(rows), OUT), file=sys.stderr)


if __name__ == "__main__":
    main()
