"""Archive discovery (FileStore::get_all / find, src/filestore/mod.rs:81-154),
mirroring src/filestore/tests.rs:16-130 on the CPU (manifest parsing only, no
device).  bfrs_batch_health_check is covered in tests/test_gpu_archive.py."""
import os

import pytest

from test_integrity import REF_FIXTURE_MANIFEST


def _setup_test_archive(tmp_path):
    # tests.rs:16-49: archive_directory/test.txt_abc123/{manifest.json, data.dat}
    root = tmp_path / "archive_directory"
    d = root / "test.txt_abc123"
    d.mkdir(parents=True)
    (d / "manifest.json").write_text(REF_FIXTURE_MANIFEST)
    (d / "data.dat").write_bytes(bytes(1000))
    return str(root)


def test_get_all_returns_files(bfrs, tmp_path):  # tests.rs:60-76
    files = bfrs.FileStore(_setup_test_archive(tmp_path)).get_all()
    assert len(files) == 1
    assert files[0]["file_name"] == "test.txt"
    assert files[0]["file_data"]["hash"] == "abc123"


def test_find_existing_file(bfrs, tmp_path):  # tests.rs:79-89
    f = bfrs.FileStore(_setup_test_archive(tmp_path)).find("test.txt")
    assert f["file_name"] == "test.txt"
    assert f["dir"].endswith("test.txt_abc123")


def test_find_nonexistent_file_fails(bfrs, tmp_path):  # tests.rs:92-100
    with pytest.raises(bfrs.BfrsError) as e:
        bfrs.FileStore(_setup_test_archive(tmp_path)).find("does_not_exist.txt")
    assert e.value.code == bfrs.E_NOT_FOUND
    assert "File 'does_not_exist.txt' not found" in str(e.value)  # mod.rs:150-153


def test_get_all_empty_archive(bfrs, tmp_path):  # tests.rs:103-113
    root = tmp_path / "empty_archive"
    root.mkdir()
    assert bfrs.FileStore(str(root)).get_all() == []


def test_all_files_returns_manifest_paths(bfrs, tmp_path):  # tests.rs:116-130
    files = bfrs.FileStore(_setup_test_archive(tmp_path)).get_all()
    assert files[0]["file_data"]["path"].endswith(os.path.join("test.txt_abc123", "manifest.json"))


def test_get_all_name_order_and_first_match(bfrs, tmp_path):
    root = tmp_path / "store"
    for dn, name, h in (("b.bin_22", "b.bin", "22"), ("a.bin_11", "a.bin", "11"),
                        ("a.bin_33", "a.bin", "33")):
        (root / dn).mkdir(parents=True)
        (root / dn / "manifest.json").write_text(
            REF_FIXTURE_MANIFEST.replace('"test.txt"', f'"{name}"').replace('"abc123"', f'"{h}"'))
    store = bfrs.FileStore(str(root))
    assert [f["dir"].rsplit("/", 1)[-1] for f in store.get_all()] == ["a.bin_11", "a.bin_33", "b.bin_22"]
    assert store.find("a.bin")["file_data"]["hash"] == "11"


def test_get_all_fails_on_an_entry_without_manifest(bfrs, tmp_path):
    # FileStore::all_files maps every entry to entry/manifest.json and get_all
    # propagates the read error (mod.rs:89-104)
    root = _setup_test_archive(tmp_path)
    os.mkdir(os.path.join(root, "half_written_computing"))
    with pytest.raises(bfrs.BfrsError):
        bfrs.FileStore(root).get_all()


def test_missing_store_root_is_an_error(bfrs, tmp_path):
    with pytest.raises(bfrs.BfrsError):
        bfrs.FileStore(str(tmp_path / "nope")).get_all()


def test_json_reports_longer_than_the_first_buffer(bfrs, tmp_path, monkeypatch):
    # the binding makes one call into a guessed buffer and a second only when
    # the report did not fit (a size query first would run a health check twice)
    store = bfrs.FileStore(_setup_test_archive(tmp_path))
    want = store.get_all()
    monkeypatch.setattr(bfrs, "_JSON_GUESS", 8)
    assert store.get_all() == want
    assert store.find(want[0]["file_name"])["dir"] == want[0]["dir"]
