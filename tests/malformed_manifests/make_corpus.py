"""Writes the malformed-manifest corpus next to this script (test data).

Each file is a manifest.json a damaged or hostile archive could hold: broken
JSON, wrong types, out-of-range numbers, missing keys, non-hex hashes, deep
nesting, shapes that disagree with the size.  Every one must come back from
bfrs_manifest_check / bfrs_store_list / bfrs_archive_stat (CPU) and from
bfrs_archive_open / bfrs_health_check / bfrs_repair (GPU) as an error code or
a clean verdict, never a crash (tests/test_malformed.py, also under ASan +
UBSan: tests/test_sanitize.py).  The `valid_*` files are the controls.

The schema is the reference's ManifestFile (src/merkle_tree/manifest.rs:12-53)
as bfrs_commit writes it (serde_json compact, sorted keys).

    python tests/malformed_manifests/make_corpus.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
H = "ab" * 32  # a 64-hex digest
S = 65536


def tier3(nseg=35, size=None):
    size = nseg * S - 100 if size is None else size
    blocks, left, b = {}, nseg, 0
    while left:
        k = min(30, left)
        blocks[str(b)] = {"segments": [H] * k, "parity": [H] * 3}
        left -= k
        b += 1
    return {"original_hash": H, "name": "big.bin", "size": size,
            "time_of_creation": "2026-01-01 00:00:00 UTC",
            "erasure_coding": {"type": "reed-solomon", "data_shards": 30, "parity_shards": 3},
            "merkle_tree": {"leaves": {str(i): H for i in range(nseg)}, "root": H,
                            "segments": {}, "blocks": blocks},
            "tier": 3, "segment_size": S}


def tier2(nseg=3):
    return {"original_hash": H, "name": "mid.bin", "size": nseg * S - 7,
            "time_of_creation": "2026-01-01 00:00:00 UTC",
            "erasure_coding": {"type": "reed-solomon", "data_shards": 1, "parity_shards": 3},
            "merkle_tree": {"leaves": {str(i): H for i in range(nseg)}, "root": H,
                            "segments": {str(i): {"data": H, "parity": [H] * 3} for i in range(nseg)},
                            "blocks": {}},
            "tier": 2, "segment_size": S}


def tier1():
    return {"original_hash": H, "name": "small.bin", "size": 1000,
            "time_of_creation": "2026-01-01 00:00:00 UTC",
            "erasure_coding": {"type": "reed-solomon", "data_shards": 1, "parity_shards": 3},
            "merkle_tree": {"leaves": {str(i): H for i in range(4)}, "root": H},
            "tier": 1, "segment_size": 0}


def dump(m):
    return json.dumps(m, separators=(",", ":"), sort_keys=True)


def edit(base, path, value=None, delete=False):
    m = json.loads(json.dumps(base))
    node = m
    for key in path[:-1]:
        node = node[key]
    if delete:
        del node[path[-1]]
    else:
        node[path[-1]] = value
    return dump(m)


def corpus():
    t3, t2, t1 = tier3(), tier2(), tier1()
    v3 = dump(t3)
    c = {
        "valid_tier3": v3, "valid_tier2": dump(t2), "valid_tier1": dump(t1),
        # broken JSON
        "empty": "", "whitespace_only": " \n\t ", "bom_prefix": "﻿" + v3,
        "truncated_10pct": v3[:len(v3) // 10], "truncated_50pct": v3[:len(v3) // 2],
        "truncated_last_byte": v3[:-1], "trailing_garbage": v3 + "xyz",
        "two_documents": v3 + v3, "not_object_array": "[]", "not_object_number": "42",
        "not_object_string": '"manifest"', "not_object_null": "null",
        "unterminated_string": '{"name": "abc', "bad_escape": '{"name": "a\\qb"}',
        "short_unicode_escape": '{"name": "\\u12"}', "bad_unicode_hex": '{"name": "\\uzzzz"}',
        "lone_high_surrogate": v3.replace('"big.bin"', '"\\ud800"'),
        "surrogate_bad_low": v3.replace('"big.bin"', '"\\ud800\\u0041"'),
        "raw_control_chars": v3.replace('"big.bin"', '"a\x01\x02\x1fb"'),
        "nul_bytes": v3.replace('"big.bin"', '"a\x00b"'),
        "missing_colon": '{"name" "x"}', "missing_comma": '{"a":1 "b":2}',
        "trailing_comma_object": '{"a":1,}', "trailing_comma_array": '{"a":[1,]}',
        "nan_literal": edit(t3, ["size"], 0).replace('"size":0', '"size":NaN'),
        "infinity_literal": edit(t3, ["size"], 0).replace('"size":0', '"size":Infinity'),
        "lone_minus": edit(t3, ["size"], 0).replace('"size":0', '"size":-'),
        "deep_arrays": "[" * 20000 + "]" * 20000,
        "deep_objects": '{"a":' * 20000 + "1" + "}" * 20000,
        "deep_in_manifest": v3[:-1] + ',"x":' + "[" * 5000 + "]" * 5000 + "}",
        # wrong types
        "size_string": edit(t3, ["size"], "2293660"),
        "size_float": edit(t3, ["size"], 0).replace('"size":0', '"size":2293660.5'),
        "size_exponent": edit(t3, ["size"], 0).replace('"size":0', '"size":1e400'),
        "tier_string": edit(t3, ["tier"], "3"), "tier_null": edit(t3, ["tier"], None),
        "segment_size_bool": edit(t3, ["segment_size"], True),
        "name_number": edit(t3, ["name"], 5), "root_array": edit(t3, ["merkle_tree", "root"], [H]),
        "blocks_array": edit(t3, ["merkle_tree", "blocks"], [t3["merkle_tree"]["blocks"]["0"]]),
        "block_segments_string": edit(t3, ["merkle_tree", "blocks", "0", "segments"], H),
        "block_parity_numbers": edit(t3, ["merkle_tree", "blocks", "0", "parity"], [1, 2, 3]),
        "erasure_coding_string": edit(t3, ["erasure_coding"], "rs"),
        "merkle_tree_null": edit(t3, ["merkle_tree"], None),
        "t2_segment_parity_string": edit(t2, ["merkle_tree", "segments", "0", "parity"], H),
        "t2_segment_data_missing": edit(t2, ["merkle_tree", "segments", "1", "data"], delete=True),
        # out-of-range numbers
        "size_negative": edit(t3, ["size"], -1),
        "size_int64_max": edit(t3, ["size"], 2**63 - 1),
        "size_int64_min": edit(t3, ["size"], -2**63),
        "size_overflow_digits": edit(t3, ["size"], 0).replace('"size":0', '"size":' + "9" * 40),
        "size_2_pow_51": edit(t3, ["size"], 2**51),
        "segment_size_zero": edit(t3, ["segment_size"], 0),
        "segment_size_negative": edit(t3, ["segment_size"], -1),
        "segment_size_one": edit(t3, ["segment_size"], 1),
        "segment_size_2_pow_40": edit(t3, ["segment_size"], 2**40),
        "segment_size_int64_max": edit(t3, ["segment_size"], 2**63 - 1),
        "tier_zero": edit(t3, ["tier"], 0), "tier_four": edit(t3, ["tier"], 4),
        "tier_negative": edit(t3, ["tier"], -3), "tier_2_pow_40": edit(t3, ["tier"], 2**40),
        "t2_segment_size_huge": edit(t2, ["segment_size"], 2**62),
        "t1_size_huge": edit(t1, ["size"], 2**62),
        "t1_size_negative": edit(t1, ["size"], -5),
        # missing keys
        **{f"missing_{k}": edit(t3, [k], delete=True)
           for k in ("original_hash", "name", "size", "tier", "segment_size", "erasure_coding",
                     "merkle_tree", "time_of_creation")},
        "missing_root": edit(t3, ["merkle_tree", "root"], delete=True),
        "missing_blocks": edit(t3, ["merkle_tree", "blocks"], delete=True),
        "missing_leaves": edit(t3, ["merkle_tree", "leaves"], delete=True),
        "missing_block_1": edit(t3, ["merkle_tree", "blocks", "1"], delete=True),
        "missing_block_parity": edit(t3, ["merkle_tree", "blocks", "0", "parity"], delete=True),
        "t2_missing_segments": edit(t2, ["merkle_tree", "segments"], delete=True),
        "t2_missing_segment_2": edit(t2, ["merkle_tree", "segments", "2"], delete=True),
        "t1_no_leaves": edit(t1, ["merkle_tree", "leaves"], {}),
        # hashes
        "root_non_hex": edit(t3, ["merkle_tree", "root"], "zz" * 32),
        "root_short": edit(t3, ["merkle_tree", "root"], "ab"),
        "root_empty": edit(t3, ["merkle_tree", "root"], ""),
        "segment_hash_non_hex": edit(t3, ["merkle_tree", "blocks", "0", "segments"],
                                     ["xyz"] + [H] * 29),
        "segment_hash_long": edit(t3, ["merkle_tree", "blocks", "1", "segments"], [H + "00"] * 5),
        "parity_hash_unicode": edit(t3, ["merkle_tree", "blocks", "0", "parity"], ["é" * 64] * 3),
        "original_hash_path": edit(t3, ["original_hash"], "../../etc/passwd"),
        "name_path_traversal": edit(t3, ["name"], "../../../tmp/x"),
        "name_huge": edit(t3, ["name"], "n" * 65536),
        # shapes that disagree with the size
        "blocks_too_few": edit(t3, ["size"], 65 * S),
        "blocks_too_many": edit(t3, ["size"], 10 * S),
        "block_31_segments": edit(t3, ["merkle_tree", "blocks", "0", "segments"], [H] * 31),
        "block_0_segments": edit(t3, ["merkle_tree", "blocks", "1", "segments"], []),
        "block_2_parity": edit(t3, ["merkle_tree", "blocks", "0", "parity"], [H] * 2),
        "block_4_parity": edit(t3, ["merkle_tree", "blocks", "0", "parity"], [H] * 4),
        "block_key_text": dump(t3).replace('"blocks":{"0":', '"blocks":{"x":'),
        "block_key_negative": dump(t3).replace('"blocks":{"0":', '"blocks":{"-1":'),
        "block_key_huge": dump(t3).replace('"blocks":{"0":', '"blocks":{"99999999999999999999":'),
        "block_key_empty": dump(t3).replace('"blocks":{"0":', '"blocks":{"":'),
        "block_keys_shifted": dump(t3).replace('"blocks":{"0":', '"blocks":{"7":'),
        "duplicate_block_key": dump(t3).replace('"blocks":{"0":', '"blocks":{"1":'),
        "duplicate_size_key": v3[:-1] + ',"size":5}',
        # integer map keys serde_json 1.0.148 refuses: it runs the JSON number
        # grammar over the raw key bytes; each would alias key 0/1
        "block_key_leading_zero": dump(t3).replace('"blocks":{"0":', '"blocks":{"01":'),
        "block_key_minus_zero": dump(t3).replace('"blocks":{"0":', '"blocks":{"-0":'),
        "block_key_escaped_digit": dump(t3).replace('"blocks":{"0":', '"blocks":{"\\u0030":'),
        "leaves_key_leading_zero": edit(t3, ["merkle_tree", "leaves"], {"00": H}),
        "leaves_key_minus_zero": edit(t3, ["merkle_tree", "leaves"], {"-0": H}),
        "t2_segment_key_leading_zero": dump(t2).replace('"segments":{"0":', '"segments":{"00":'),
        "leaves_gap": edit(t3, ["merkle_tree", "leaves"], {"0": H, "5": H}),
        "leaves_key_text": edit(t3, ["merkle_tree", "leaves"], {"a": H}),
        "t2_segment_count_short": edit(t2, ["size"], 9 * S),
        "t2_segment_4_parity": edit(t2, ["merkle_tree", "segments", "0", "parity"], [H] * 4),
        "t2_segment_keys_shifted": dump(t2).replace('"segments":{"0":', '"segments":{"9":'),
        "many_blocks": edit(t3, ["merkle_tree", "blocks"],
                            {str(b): {"segments": [H] * 30, "parity": [H] * 3} for b in range(100)}),
        "zero_size_tier3": edit(edit_obj(t3, ["merkle_tree", "blocks"], {}), ["size"], 0),
    }
    return c


def edit_obj(base, path, value):
    return json.loads(edit(base, path, value))


def main():
    for name in os.listdir(HERE):
        if name.endswith(".json"):
            os.unlink(os.path.join(HERE, name))
    for name, text in corpus().items():
        with open(os.path.join(HERE, name + ".json"), "w", encoding="utf-8",
                  errors="surrogatepass") as f:
            f.write(text)
    print(len(corpus()), "files")


if __name__ == "__main__":
    main()
