#!/usr/bin/env python3
"""Writes tests/golden/tf_dtype_map.json: the reference's TF dtype map
(srcs/cpp/include/kungfu/tensorflow/ops.h to_kungfu_type) with the KungFu codes
of srcs/cpp/include/kungfu/dtype.h, read from the reference's headers as text.

  python tests/golden/gen_tf_dtype_map.py [/root/reference]
"""
import json
import os
import re
import sys

# TF DataType enum names -> the dtype names TF reports (tf.float32.name, ...)
TF_NAMES = {"INT32": "int32", "INT64": "int64", "BFLOAT16": "bfloat16", "HALF": "float16",
            "FLOAT": "float32", "DOUBLE": "float64", "BOOL": "bool"}


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    inc = os.path.join(ref, "srcs", "cpp", "include", "kungfu")
    with open(os.path.join(inc, "dtype.h")) as f:
        codes = {m.group(1): (int(m.group(2)) << 16) | (int(m.group(3)) << 8) | 8
                 for m in re.finditer(r"KungFu_(\w+)\s*=\s*TYPE_CODE\((\d+),\s*(\d+)\)", f.read())}
    with open(os.path.join(inc, "tensorflow", "ops.h")) as f:
        src = f.read()
    body = src[src.index("to_kungfu_type"):]
    body = body[:body.index("default:")]
    table = {TF_NAMES[m.group(1)]: {"kungfu": "KungFu_" + m.group(2), "code": codes[m.group(2)]}
             for m in re.finditer(r"case DT_(\w+):\s*return KungFu_(\w+);", body)}
    out = {"source": "srcs/cpp/include/kungfu/tensorflow/ops.h to_kungfu_type; codes from "
                     "srcs/cpp/include/kungfu/dtype.h; other dtypes throw "
                     "std::invalid_argument(\"unsupported dtype\")",
           "map": table}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tf_dtype_map.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(path, table)


if __name__ == "__main__":
    main()
