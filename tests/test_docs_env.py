"""docs/environment.md lists exactly the environment knobs the code reads (round-5 verdict: the
table had drifted -- removed GEMM variants still documented, new knobs missing)."""
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1]
_C = re.compile(r'(?:getenv(?:_flag_off|_flag)?|env_int)\("([A-Z][A-Z0-9_]+)"')
_PY = re.compile(r'(?:environ(?:\.get|\.setdefault)?[\[(]|getenv\()"([A-Z][A-Z0-9_]+)"')
# read by the code but owned by the runtime / shell, not knobs of this framework
_EXTERNAL = {"TERM", "HOME", "RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "GPU_MAX_HW_QUEUES",
             "HSA_ENABLE_IPC_MODE_LEGACY", "PYTORCH_ROCM_ARCH", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
             "CUDA_VISIBLE_DEVICES", "TMPDIR", "OMP_NUM_THREADS", "MAX_JOBS", "GRAFT_REPO_ROOT", "USER", "PATH",
             "LD_LIBRARY_PATH", "PYTHONPATH", "XDG_RUNTIME_DIR", "ROCM_PATH", "HIPCC", "CXX", "CC", "NPROC"}


def _code_knobs():
    names = set()
    for p in (ROOT / "libsplinter_amd" / "csrc").rglob("*"):
        if p.suffix in (".hip", ".cpp", ".hpp", ".h", ".c"):
            names |= set(_C.findall(p.read_text(errors="replace")))
    pys = list((ROOT / "libsplinter_amd").rglob("*.py")) + list((ROOT / "scripts").glob("*.py"))
    pys += [ROOT / "bench.py", ROOT / "__graft_entry__.py"]
    for p in pys:
        if p.exists():
            names |= set(_PY.findall(p.read_text(errors="replace")))
    return {n for n in names if n not in _EXTERNAL and not n.startswith(("HSA_", "HIP_", "ROC", "TORCH", "NCCL_"))}


def _doc_knobs():
    text = (ROOT / "docs" / "environment.md").read_text()
    return set(re.findall(r"`([A-Z][A-Z0-9_]+)(?:=[^`]*)?`", text))


def test_every_knob_the_code_reads_is_documented():
    missing = sorted(_code_knobs() - _doc_knobs())
    assert not missing, f"undocumented environment knobs: {missing}"


def test_documented_library_knobs_are_read_somewhere():
    text = (ROOT / "docs" / "environment.md").read_text()
    lib = text[:text.index("## CLI")]
    documented = set(re.findall(r"^\| `([A-Z][A-Z0-9_]+)` \|", lib, re.M))
    stale = sorted(documented - _code_knobs())
    assert not stale, f"documented knobs no code reads: {stale}"
