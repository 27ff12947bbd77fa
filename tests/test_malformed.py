"""CPU: the malformed-manifest corpus (tests/malformed_manifests, written by
make_corpus.py) through the host-side entry points that parse on-disk
manifests: bfrs_manifest_check (ManifestFile::new + validate,
src/merkle_tree/manifest.rs:47-88), bfrs_store_list / bfrs_store_find
(FileStore::get_all / find, src/filestore/mod.rs:81-154) and
bfrs_archive_stat (the mount's getattr geometry,
src/mount/filesystem_unix.rs:153-174).  Every file must come back as a result
or a BfrsError with an error code -- never a crash, a hang or another
exception.  tests/test_sanitize.py runs this file again under ASan + UBSan;
the GPU entry points (archive open / health check / repair) take the same
corpus in tests/test_gpu_archive.py."""
import glob
import os

import pytest

CORPUS = os.path.join(os.path.dirname(__file__), "malformed_manifests")
FILES = sorted(glob.glob(os.path.join(CORPUS, "*.json")))

# must parse, validate and give a geometry (the controls)
VALID = {"valid_tier1", "valid_tier2", "valid_tier3"}
# the geometry check refuses these (bounds, tier, shape vs size)
GEOMETRY_ERRORS = {
    "size_negative", "size_int64_max", "size_int64_min", "size_2_pow_51",
    "segment_size_zero", "segment_size_one", "segment_size_2_pow_40",
    "segment_size_int64_max", "tier_zero", "tier_four",
    "t2_segment_size_huge", "t1_size_huge", "t1_size_negative", "missing_blocks",
    "missing_block_1", "blocks_too_few", "blocks_too_many", "block_31_segments",
    "block_0_segments", "block_2_parity", "block_4_parity", "block_keys_shifted",
    "duplicate_block_key", "t2_missing_segments", "t2_missing_segment_2",
    "t2_segment_count_short", "t2_segment_4_parity", "t2_segment_keys_shifted", "many_blocks",
}
# the parser refuses these, as serde_json::from_str into ManifestFile would
# (not JSON, wrong types or ranges, missing required fields, duplicate fields)
PARSE_ERRORS = {
    "empty", "whitespace_only", "bom_prefix", "truncated_10pct", "truncated_50pct",
    "truncated_last_byte", "trailing_garbage", "two_documents", "not_object_array",
    "not_object_number", "not_object_string", "not_object_null", "unterminated_string",
    "bad_escape", "short_unicode_escape", "bad_unicode_hex", "missing_colon", "missing_comma",
    "trailing_comma_object", "trailing_comma_array", "nan_literal", "infinity_literal",
    "deep_arrays", "deep_objects", "deep_in_manifest", "size_string", "tier_string",
    "tier_null", "segment_size_bool", "name_number", "root_array", "blocks_array",
    "block_segments_string", "block_parity_numbers", "erasure_coding_string",
    "merkle_tree_null", "t2_segment_parity_string", "t2_segment_data_missing",
    "missing_original_hash", "missing_name", "missing_size", "missing_tier",
    "missing_segment_size", "missing_erasure_coding", "missing_merkle_tree", "missing_root",
    "block_key_text", "block_key_huge", "block_key_empty", "missing_block_parity",
    "leaves_key_text", "duplicate_size_key", "size_float", "size_exponent", "lone_minus",
    "size_overflow_digits", "segment_size_negative", "tier_2_pow_40", "tier_negative",
    "block_key_negative", "missing_time_of_creation", "nul_bytes", "raw_control_chars",
    "lone_high_surrogate", "surrogate_bad_low",
    "block_key_leading_zero", "block_key_minus_zero", "block_key_escaped_digit",
    "leaves_key_leading_zero", "leaves_key_minus_zero", "t2_segment_key_leading_zero",
}


def _name(path):
    return os.path.basename(path)[:-5]


def test_corpus_is_present_and_classified():
    names = {_name(p) for p in FILES}
    assert len(names) >= 100
    assert VALID <= names and GEOMETRY_ERRORS <= names and PARSE_ERRORS <= names
    assert not (GEOMETRY_ERRORS & PARSE_ERRORS)


@pytest.mark.parametrize("path", FILES, ids=_name)
def test_manifest_check_never_crashes(bfrs, path):
    raw = open(path, "rb").read()
    name = _name(path)
    try:
        valid, canon = bfrs.manifest_check(raw)
    except bfrs.BfrsError as e:
        assert e.code == bfrs.E_WRAPPER, (name, e.code)
        assert name in PARSE_ERRORS, (name, str(e))
        return
    assert name not in PARSE_ERRORS, name
    if name in VALID:
        assert valid, name
        # the canonical form parses to the same manifest
        assert bfrs.manifest_check(canon)[1] == canon


@pytest.mark.parametrize("path", FILES, ids=_name)
def test_archive_stat_and_store_never_crash(bfrs, path, tmp_path):
    name = _name(path)
    adir = tmp_path / "store" / f"{name}_{'ab' * 32}"
    adir.mkdir(parents=True)
    (adir / "manifest.json").write_bytes(open(path, "rb").read())
    try:
        st = bfrs.archive_stat(str(adir))
    except bfrs.BfrsError as e:
        assert e.code == bfrs.E_WRAPPER, (name, e.code)
        assert name in PARSE_ERRORS or name in GEOMETRY_ERRORS, (name, str(e))
    else:
        assert name not in PARSE_ERRORS and name not in GEOMETRY_ERRORS, (name, st)
        assert 1 <= st["tier"] <= 3 and st["segments"] >= 1 or st["size"] == 0
    store = bfrs.FileStore(str(tmp_path / "store"))
    try:
        files = store.get_all()
    except bfrs.BfrsError as e:  # get_all fails on a manifest that does not parse
        assert e.code == bfrs.E_WRAPPER, (name, e.code)
        assert name in PARSE_ERRORS, (name, str(e))
    else:
        assert name not in PARSE_ERRORS, name
        assert len(files) == 1


def test_valid_controls_geometry(bfrs, tmp_path):
    """The controls' geometry: tier 3 = 35 segments of 64 KiB in 2 blocks
    (30 + 5); tier 2 = 3 segments; tier 1 = one 1000-byte segment."""
    want = {"valid_tier3": dict(tier=3, size=35 * 65536 - 100, segment_size=65536, segments=35,
                                blocks=2),
            "valid_tier2": dict(tier=2, size=3 * 65536 - 7, segment_size=65536, segments=3, blocks=0),
            "valid_tier1": dict(tier=1, size=1000, segment_size=0, segments=1, blocks=0)}
    for name, w in want.items():
        d = tmp_path / name
        d.mkdir()
        (d / "manifest.json").write_bytes(open(os.path.join(CORPUS, name + ".json"), "rb").read())
        assert bfrs.archive_stat(str(d)) == w


def test_archive_stat_missing_manifest(bfrs, tmp_path):
    with pytest.raises(bfrs.BfrsError) as e:
        bfrs.archive_stat(str(tmp_path / "nope"))
    assert e.value.code == bfrs.E_WRAPPER
