"""ctypes binding of libmetacov_amd.so (declared in include/metacov_amd.h).

The shared library is built in-tree (`python -m metacov_amd.build`) and is
the ONLY compute path: there is no CPU fallback.  A missing library raises
`LibraryNotBuilt`; a ctx on a machine without a HIP device raises
`MetacovError` from `mc_ctx_create`.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("METACOV_AMD_LIB", os.path.join(HERE, "libmetacov_amd.so"))

MC_OK = 0
MC_E_INVALID = -1
MC_E_HIP = -2
MC_E_IO = -3
MC_E_STATE = -4
MC_E_RANGE = -5


class MetacovError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (code %d)" % (msg, code))
        self.code = code


class LibraryNotBuilt(ImportError):
    pass


class RegionStat(ctypes.Structure):
    """mc_region_stat (72 bytes)."""
    _fields_ = [("n", ctypes.c_int64), ("sum", ctypes.c_int64), ("sumsq", ctypes.c_uint64),
                ("min", ctypes.c_int64), ("max", ctypes.c_int64),
                ("med_lo", ctypes.c_int64), ("med_hi", ctypes.c_int64),
                ("q23_sum", ctypes.c_int64), ("q23_cnt", ctypes.c_int64)]


class ScanConfig(ctypes.Structure):
    """mc_scan_config."""
    _fields_ = [("n_flags", ctypes.c_int32), ("flags", ctypes.c_uint32 * 16),
                ("base_on", ctypes.c_int32), ("base_start", ctypes.c_int32),
                ("kmer_on", ctypes.c_int32), ("kmer_k", ctypes.c_int32),
                ("kmer_nk", ctypes.c_int32), ("kmer_step", ctypes.c_int32),
                ("kmer_offset", ctypes.c_int32),
                ("mirror_on", ctypes.c_int32), ("mirror_offset", ctypes.c_int32),
                ("mirror_n", ctypes.c_int32), ("isize_on", ctypes.c_int32)]


class Timings(ctypes.Structure):
    _fields_ = [("cigar_ms", ctypes.c_float), ("depth_ms", ctypes.c_float),
                ("stats_ms", ctypes.c_float), ("prepare_ms", ctypes.c_float),
                ("depth_launches", ctypes.c_int64), ("stats_launches", ctypes.c_int64),
                ("fused_depth_ms_total", ctypes.c_double), ("fused_stats_ms_total", ctypes.c_double),
                ("fused_calls", ctypes.c_int64), ("direct_batches", ctypes.c_int64),
                ("full_prepares", ctypes.c_int64), ("prepare_ms_total", ctypes.c_double),
                ("halo_redos", ctypes.c_int64), ("direct_halo", ctypes.c_int64)]


class GpuDecodeTimings(ctypes.Structure):
    """mc_bam_gpu_timings."""
    _fields_ = [("read_ms", ctypes.c_double), ("inflate_ms", ctypes.c_double),
                ("parse_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("windows", ctypes.c_int64), ("blocks", ctypes.c_int64), ("resyncs", ctypes.c_int64),
                ("compressed_bytes", ctypes.c_int64), ("inflated_bytes", ctypes.c_int64),
                ("scan_ms", ctypes.c_double), ("upload_ms", ctypes.c_double), ("kernel_ms", ctypes.c_double),
                ("open_ms", ctypes.c_double), ("parse_rounds", ctypes.c_int64),
                ("resync_passes", ctypes.c_int64)]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_U32 = ctypes.c_uint32
_PI32 = ctypes.POINTER(ctypes.c_int32)
_PI64 = ctypes.POINTER(ctypes.c_int64)
_PU32 = ctypes.POINTER(ctypes.c_uint32)
_PP = ctypes.POINTER(ctypes.c_void_p)

# name -> argtypes (all return int unless listed in _RESTYPE)
SIGNATURES = {
    "mc_last_error": [],
    "mc_version": [],
    "mc_build_id": [],
    "mc_runtime_init": [ctypes.c_int],
    "mc_ctx_create": [ctypes.c_int, _PP],
    "mc_ctx_destroy": [_P],
    "mc_ctx_set_stream": [_P, _P],
    "mc_ctx_device": [_P, ctypes.POINTER(ctypes.c_int)],
    "mc_set_contigs": [_P, _I32, _P],
    "mc_add_reads": [_P, _I64, _P, _P, _P],
    "mc_add_reads_device": [_P, _I64, _P, _P, _P],
    "mc_add_reads_async": [_P, _I64, _P, _P, _P],
    "mc_pinned_alloc": [_I64, _PP],
    "mc_pinned_free": [_P],
    "mc_add_reads_cigar": [_P, _I64, _P, _P, _P, _P],
    "mc_add_reads_cigar_device": [_P, _I64, _P, _P, _P, _P],
    "mc_clear_reads": [_P],
    "mc_invalidate": [_P],
    "mc_set_direct_prepare": [_P, ctypes.c_int],
    "mc_set_legacy_endpos": [_P, ctypes.c_int],
    "mc_prepare": [_P],
    "mc_compute_depth": [_P],
    "mc_get_depth": [_P, _I32, _I64, _I64, _P],
    "mc_depth_device": [_P, _PP, _PI64],
    "mc_contig_offset": [_P, _I32, _PI64, _PI64],
    "mc_region_stats": [_P, _I64, _P, _P, _P, _P],
    "mc_region_stats_device": [_P, _I64, _P, _P, _P, _P],
    "mc_region_np_sqdev": [_P, _I64, _P, _P, _P, _P, _P],
    "mc_compute_depth_stats": [_P, _I64, _P, _P, _P, _P],
    "mc_compute_depth_stats_device": [_P, _I64, _P, _P, _P, _P],
    "mc_fused_fallbacks": [_P, _PI64],
    "mc_fused_recomputes": [_P, _PI64],
    "mc_aligned_bases": [_P, _PI64],
    "mc_max_depth": [_P, _PI32],
    "mc_get_timings": [_P, ctypes.POINTER(Timings)],
    "mc_synchronize": [_P],
    "mc_depth_cap_mask": [_I64, _P, _P, _P, _I32, ctypes.c_int, _P, _PI64],
    "mc_depth_cap_mask_device": [ctypes.c_int, _I64, _P, _P, _P, _I32, _P, _PI64],
    "mc_add_reads_capped": [_P, _I64, _P, _P, _P, _I64, _P, _P, _P, _I32, _PI64],
    "mc_bam_open": [ctypes.c_char_p, ctypes.c_int, _U32, ctypes.c_int, _PP],
    "mc_bam_close": [_P],
    "mc_bam_n_targets": [_P, _PI32],
    "mc_bam_target": [_P, _I32, ctypes.POINTER(ctypes.c_char_p), _PI64],
    "mc_bam_counts": [_P, _PI64, _PI64, _PI64, _PI64],
    "mc_bam_intervals": [_P, _P, _P, _P],
    "mc_bam_n_cigar_words": [_P, _PI64],
    "mc_bam_cigars": [_P, _P, _P],
    "mc_bam_stream_open": [ctypes.c_char_p, ctypes.c_int, _U32, _I64, _PP],
    "mc_bam_stream_next": [_P, _I64, _P, _P, _P, _PI64],
    "mc_bam_stream_header": [_P, _PP],
    "mc_bam_stream_close": [_P],
    "mc_bam_index_build": [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int],
    "mc_bam_index_stats": [ctypes.c_char_p, _I32, _P, _P, _PI64],
    "mc_bam_open_contigs": [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, _U32, ctypes.c_int, _I32,
                            _P, _PP],
    "mc_bam_write": [ctypes.c_char_p, _I32, _P, _P, _I64, _P, _P, _P, _P, _P, _I32, ctypes.c_int,
                     ctypes.c_int],
    "mc_bam_gpu_open": [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, _U32, _I64, _PP],
    "mc_bam_gpu_header": [_P, _PP],
    "mc_bam_gpu_intervals_device": [_P, _PI64, _PP, _PP, _PP],
    "mc_bam_gpu_intervals": [_P, _P, _P, _P],
    "mc_bam_gpu_stats": [_P, _P],
    "mc_bam_gpu_close": [_P],
    "mc_bam_gpu_trim": [_P, _PI64],
    "mc_bam_gpu_open_scan": [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, _I64, _PP],
    "mc_bam_gpu_scan_device": [_P, _PI64, _PP, _PP, _PP, _PP, _PP, _PP, _PP, _PI64],
    "mc_bam_gpu_open_reads": [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _I64, _PP],
    "mc_bam_gpu_reads_device": [_P, _PI64, _PP, _PP, _PP, _PP, _PP, _PP, _PP, _PP, _PP, _PI64],
    "mc_bam_gpu_reads_copy": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "mc_bam_gpu_open_reads_extents": [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _I32, _P, _I64,
                                      _I32, _P, _PP],
    "mc_bam_index_extents": [ctypes.c_char_p, _I32, _P, _PI64],
    "mc_bam_gpu_open_contigs": [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, _U32, _I32, _P,
                                _PP],
    "mc_bam_gpu_open_extents": [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, _U32, _I32, _P, _I64, _I32, _P,
                                _PP],
    "mc_bam_gpu_extents": [_P, _I32, _P, _PI64],
    "mc_bam_gpu_restrict": [_P, _I32, _P],
    "mc_bam_gpu_intervals_range": [_P, _I64, _I64, _P, _P, _P],
    "mc_gz_inflate_host": [_P, _I64, _P, _I64],
    "mc_bam_rec_parse_host": [_P, _I64, _I32, _U32, _P],
    "mc_bam_rec_chain_host": [_P, _I64, _I64, _I32, ctypes.c_int],
    "mc_bgzf_scan_host": [ctypes.c_char_p, ctypes.c_int, _PI64, _PI64, _PI64, _I64],
    # pileup.experimental: read side (host) and sequence side (GPU)
    "mc_reads_open": [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, _PP],
    "mc_reads_open_gpu": [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _PP],
    "mc_reads_open_gpu_extents": [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _I32, _P, _I64, _I32,
                                  _P, _PP],
    "mc_reads_fields": [_P, _PP, _PP, _PP, _PP, _PP, _PP, _PP, _PP, _PI64, _PP, _PP],
    "mc_reads_close": [_P],
    "mc_reads_header": [_P, _PI32, _PI64, _PI64],
    "mc_reads_target": [_P, _I32, ctypes.POINTER(ctypes.c_char_p), _PI64],
    "mc_experimental_reads": [_P, ctypes.c_int, _P, _P, _P, _P, _I64, _P, _P, _P, ctypes.c_int,
                              _P, _P],
    "mc_experimental_events": [_P, _I64, _I64, _P, _PI64],
    "mc_ecor_create": [ctypes.c_int, _PP],
    "mc_ecor_destroy": [_P],
    "mc_ecor_set_sequence": [_P, _I64, _P],
    "mc_ecor_set_tables": [_P, ctypes.c_int, _P, _P, ctypes.c_int, _P],
    "mc_ecor_run": [_P, _I64, _P, _P, _P, _P, _P, _P, ctypes.POINTER(ctypes.c_float)],
    # metacov scan: read sources (host) and histograms (GPU)
    "mc_scan_src_open_bam": [ctypes.c_char_p, ctypes.c_int, _PP],
    "mc_scan_src_open_fastq": [ctypes.c_char_p, ctypes.c_char_p, _PP],
    "mc_scan_src_open_sam": [ctypes.c_char_p, _PP],
    "mc_scan_src_close": [_P],
    "mc_scan_src_n_targets": [_P, _PI32],
    "mc_scan_src_target": [_P, _I32, ctypes.POINTER(ctypes.c_char_p), _PI64],
    "mc_scan_src_next": [_P, _I64, _I64, _PI64],
    "mc_scan_src_batch": [_P, _PP, _PP, _PP, _PP, _PP, _PP, _PP, _PI64],
    "mc_scan_src_records": [_P, _PI64],
    "mc_scan_create": [ctypes.c_int, _P, _PP],
    "mc_scan_destroy": [_P],
    "mc_scan_set_reference": [_P, _I32, _P, _P, _I64, _P],
    "mc_scan_add_batch": [_P, _I64, _P, _P, _P, _P, _P, _P, _P],
    "mc_scan_add_batch_device": [_P, _I64, _P, _P, _P, _P, _P, _P, _P, _I32, _I64,
                                 ctypes.POINTER(ctypes.c_float)],
    "mc_scan_run": [_P, _P, _I32, _P, _I64, _I64, _PI64],
    "mc_scan_run_gpu": [_P, _P, _I32, _P, _I64, _PI64],
    "mc_scan_dims": [_P, _PI32, _PI64, _PI64, _PI32, _PI64],
    "mc_scan_results": [_P, _P, _P, _P, _P, _P],
    "mc_scan_timing": [_P, ctypes.POINTER(ctypes.c_float), _PI64],
}
_RESTYPE = {"mc_last_error": ctypes.c_char_p, "mc_version": ctypes.c_char_p,
            "mc_build_id": ctypes.c_char_p}

_lib = None
_variants = {}


def load(path=None):
    """Loads the library once; raises LibraryNotBuilt if it is absent.
    `path` loads another build of the same ABI side by side (A/B runs)."""
    global _lib
    if path is not None and path != LIB_PATH:
        if path not in _variants:
            _variants[path] = _open(path, partial=True)
        return _variants[path]
    if _lib is None:
        _lib = _open(LIB_PATH)
    return _lib


def _share_torch_hip_runtime():
    """Loads PyTorch's bundled HIP runtime (soname libamdhip64.so.7, as the
    library's own dependency) before the library, so both use one runtime in
    any import order.  Loaded the other way round, /opt/rocm's runtime came
    first and a later `import torch` found no device (hipErrorNoDevice) in
    the same process.  No-op without torch."""
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        hip = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(hip):
            ctypes.CDLL(hip, mode=ctypes.RTLD_GLOBAL)
            return


def _open(path, partial=False):
    """partial: an A/B build of an older revision may lack newer entry points."""
    if not os.path.exists(path):
        raise LibraryNotBuilt(
            "%s not found: build it with `python -m metacov_amd.build` "
            "(hipcc --offload-arch=gfx950). metacov_amd has no CPU fallback." % path)
    _share_torch_hip_runtime()
    lib = ctypes.CDLL(path)
    for name, argtypes in SIGNATURES.items():
        if partial and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPE.get(name, ctypes.c_int)
    return lib


def check(rc, lib=None):
    if rc != MC_OK:
        msg = (lib or load()).mc_last_error()
        raise MetacovError(rc, msg.decode() if msg else "error")
    return rc


def ptr(arr):
    """ctypes pointer of a C-contiguous numpy array."""
    return ctypes.c_void_p(arr.ctypes.data) if arr is not None and arr.size else None
