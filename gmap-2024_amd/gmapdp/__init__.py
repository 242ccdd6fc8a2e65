"""gmapdp -- Python host binding of libgmapdp.so (the MI355X Dynprog engine).

Mirrors the reference's Dynprog_* operator interface for tests and the bench:
argument names and meaning follow dynprog_single.c:429 (Dynprog_single_gap),
results follow its out-parameters and the List_T of Pair_T it returns.

The native library is required: importing this module on a machine without
the built extension, or calling into it without a HIP device, raises -- there
is no CPU fallback on the product path.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# GMAPDP_LIB: an alternative build of the library (experiments); the default is the in-tree one
LIB_PATH = os.environ.get("GMAPDP_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libgmapdp.so")

WATSON, JUMP_LATE, WIDEBAND = 0x1, 0x2, 0x4
DEVICE = "device"  # splice / candidate probabilities evaluated by the engine's device MaxEnt (a NULL arena)
CTX_ONE_STREAM, CTX_PRIO_HIGH, CTX_PRIO_LOW, CTX_BLOCKING_SYNC, CTX_POLL_SYNC = 0x1, 0x2, 0x4, 0x8, 0x10  # create_ex flags
CTX_TWO_SIDES = 0x20
SIMD = 0x40  # GMAPDP_SIMD: the reference's SIMD builds' semantics (every problem family)
HALFP, FINALP = 0x8, 0x10
KNOWN_SITES = 0x80  # GMAPDP_KNOWN_SITES: known splice sites of a genome gap (gmap -s)
UNSET = -2147483648
NEG_INFINITY_32 = -32768
MAX_RLENGTH, MAX_GLENGTH = 660, 2000


class GmapdpError(RuntimeError):
    pass


class SingleProblem(C.Structure):
    _fields_ = [("qoff", C.c_int32), ("rlength", C.c_int32), ("glength", C.c_int32), ("roffset", C.c_int32),
                ("goffset", C.c_int32), ("chroffset", C.c_uint64), ("chrhigh", C.c_uint64), ("flags", C.c_int32),
                ("genestrand", C.c_int32), ("extraband", C.c_int32), ("defect_rate", C.c_double),
                ("dynprogindex", C.c_int32), ("pad_", C.c_int32)]


class EndProblem(C.Structure):
    _fields_ = [("qoff", C.c_int32), ("rlength", C.c_int32), ("glength", C.c_int32), ("roffset", C.c_int32),
                ("goffset", C.c_int32), ("chroffset", C.c_uint64), ("chrhigh", C.c_uint64), ("flags", C.c_int32),
                ("genestrand", C.c_int32), ("extraband", C.c_int32), ("end3p", C.c_int32), ("endalign", C.c_int32),
                ("require_pos_score_p", C.c_int32), ("dynprogindex", C.c_int32), ("defect_rate", C.c_double)]


class Result(C.Structure):
    _fields_ = [("npairs", C.c_int32), ("pair_offset", C.c_int32), ("traceback_score", C.c_int32),
                ("nmatches", C.c_int32), ("nmismatches", C.c_int32), ("nopens", C.c_int32),
                ("nindels", C.c_int32), ("dynprogindex", C.c_int32)]


class GenomeProblem(C.Structure):
    _fields_ = [("qoff", C.c_int32), ("rlength", C.c_int32), ("glengthL", C.c_int32), ("glengthR", C.c_int32),
                ("roffset", C.c_int32), ("goffsetL", C.c_int32), ("rev_goffsetR", C.c_int32),
                ("chroffset", C.c_uint64), ("chrhigh", C.c_uint64), ("flags", C.c_int32),
                ("cdna_direction", C.c_int32), ("genestrand", C.c_int32), ("extraband", C.c_int32),
                ("maxpeelback", C.c_int32), ("dynprogindex", C.c_int32), ("known_offset", C.c_int32),
                ("defect_rate", C.c_double), ("prob_offset", C.c_int64)]


class GenomeResult(C.Structure):
    _fields_ = [("npairs", C.c_int32), ("pair_offset", C.c_int32), ("traceback_score", C.c_int32),
                ("nmatches", C.c_int32), ("nmismatches", C.c_int32), ("nopens", C.c_int32),
                ("nindels", C.c_int32), ("dynprogindex", C.c_int32), ("new_leftgenomepos", C.c_int32),
                ("new_rightgenomepos", C.c_int32), ("exonhead", C.c_int32), ("introntype", C.c_int32),
                ("gap_index", C.c_int32), ("gap_queryjump", C.c_int32), ("left_prob", C.c_double),
                ("right_prob", C.c_double)]


class CdnaProblem(C.Structure):
    _fields_ = [("qoffL", C.c_int32), ("qoffR", C.c_int32), ("rlengthL", C.c_int32), ("rlengthR", C.c_int32),
                ("glength", C.c_int32), ("roffsetL", C.c_int32), ("rev_roffsetR", C.c_int32), ("goffset", C.c_int32),
                ("chroffset", C.c_uint64), ("chrhigh", C.c_uint64), ("flags", C.c_int32), ("genestrand", C.c_int32),
                ("extraband", C.c_int32), ("dynprogindex", C.c_int32), ("defect_rate", C.c_double)]


class CdnaResult(C.Structure):
    _fields_ = [("npairs", C.c_int32), ("pair_offset", C.c_int32), ("traceback_score", C.c_int32),
                ("dynprogindex", C.c_int32), ("incompletep", C.c_int32), ("gap_index", C.c_int32),
                ("gap_queryjump", C.c_int32), ("pad_", C.c_int32)]


class SjProblem(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("qoff", "joff", "rlength", "glength", "roffset", "goffset_anchor",
                                         "goffset_far", "contlength", "flags", "genestrand", "extraband", "end3p",
                                         "dynprogindex", "pad_")] + [("defect_rate", C.c_double)]


class SjResult(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("npairs", "pair_offset", "traceback_score", "missscore", "nmatches",
                                         "nmismatches", "nopens", "nindels", "dynprogindex", "known_index")]


class OligoProblem(C.Structure):
    _fields_ = [("qoff", C.c_int32), ("querylength", C.c_int32), ("chrstart", C.c_uint32), ("chrend", C.c_uint32),
                ("chroffset", C.c_uint64), ("chrhigh", C.c_uint64), ("plusp", C.c_int32), ("minor", C.c_int32)]


class OligoResult(C.Structure):
    _fields_ = [("totalpositions", C.c_int32), ("maxnconsecutive", C.c_int32), ("oned_matrix_p", C.c_int32),
                ("ndiagonals", C.c_int32), ("table_offset", C.c_int64), ("diag_offset", C.c_int64)]


class Stage2Problem(C.Structure):
    _fields_ = [("qoff", C.c_int32), ("querylength", C.c_int32), ("chrstart", C.c_uint32), ("chrend", C.c_uint32),
                ("chroffset", C.c_uint64), ("chrhigh", C.c_uint64), ("plusp", C.c_int32), ("splicingp", C.c_int32),
                ("maxintronlen", C.c_int32), ("pad_", C.c_int32)]


class Stage2Result(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("nresults", "npaths", "ncovered", "status", "diag_querystart",
                                          "diag_queryend", "path_offset", "npairs")]


class MicroexonProblem(C.Structure):
    _fields_ = [("qoff", C.c_int32), ("rlength", C.c_int32), ("roffset", C.c_int32), ("goffsetL", C.c_int32),
                ("rev_goffsetR", C.c_int32), ("cdna_direction", C.c_int32), ("chroffset", C.c_uint64),
                ("chrhigh", C.c_uint64), ("watsonp", C.c_int32), ("genestrand", C.c_int32),
                ("dynprogindex", C.c_int32), ("pad_", C.c_int32)]


class MicroexonCandidate(C.Structure):
    _fields_ = [("cL", C.c_int32), ("cR", C.c_int32), ("candidate", C.c_int32), ("middlelength", C.c_int32),
                ("pos2", C.c_uint64), ("pos3", C.c_uint64), ("model2", C.c_int32), ("model3", C.c_int32)]
MICROEXON_RESULT_DTYPE = np.dtype([("ncandidates", "<i4"), ("dynprogindex", "<i4"), ("microintrontype", "<i4"),
                                   ("npairs", "<i4"), ("cand_offset", "<i8"), ("pair_offset", "<i8"),
                                   ("bestprob2", "<f8"), ("bestprob3", "<f8")])


_CFMT = {C.c_int32: "<i4", C.c_uint32: "<u4", C.c_int64: "<i8", C.c_uint64: "<u8", C.c_double: "<f8"}


def _struct_dtype(S, fmt=None):
    """numpy view of a ctypes structure (field formats from the ctypes types unless given)."""
    fmt = fmt or [_CFMT[t] for _, t in S._fields_]
    return np.dtype({"names": [n for n, _ in S._fields_], "formats": fmt,
                     "offsets": [S.__dict__[n].offset for n, _ in S._fields_], "itemsize": C.sizeof(S)})


GENOME_PROBLEM_DTYPE = _struct_dtype(GenomeProblem)
GENOME_RESULT_DTYPE = _struct_dtype(GenomeResult)
CDNA_PROBLEM_DTYPE = _struct_dtype(CdnaProblem)
CDNA_RESULT_DTYPE = _struct_dtype(CdnaResult)
SJ_PROBLEM_DTYPE = _struct_dtype(SjProblem)
SJ_RESULT_DTYPE = _struct_dtype(SjResult)
OLIGO_PROBLEM_DTYPE = _struct_dtype(OligoProblem)
OLIGO_RESULT_DTYPE = _struct_dtype(OligoResult)
STAGE2_PROBLEM_DTYPE = _struct_dtype(Stage2Problem)
STAGE2_RESULT_DTYPE = _struct_dtype(Stage2Result)
PATH_DTYPE = np.dtype([("pair_offset", "<i8"), ("npairs", "<i4"), ("pad_", "<i4")])
PATH_PAIR_DTYPE = np.dtype([("querypos", "<i4"), ("genomepos", "<i4"), ("queryjump", "<i4"), ("genomejump", "<i4"),
                            ("cdna", "S1"), ("comp", "S1"), ("genome", "S1"), ("genomealt", "S1")])

PAIR_DTYPE = np.dtype([("querypos", "<i4"), ("genomepos", "<i4"), ("jump", "<i4"), ("cdna", "S1"),
                       ("comp", "S1"), ("genome", "S1"), ("genomealt", "S1")])
RESULT_DTYPE = np.dtype([(n, "<i4") for n, _ in Result._fields_])
PROBLEM_DTYPE = _struct_dtype(SingleProblem)
MICROEXON_PROBLEM_DTYPE = _struct_dtype(MicroexonProblem)
MICROEXON_CANDIDATE_DTYPE = _struct_dtype(MicroexonCandidate)
END_PROBLEM_DTYPE = _struct_dtype(EndProblem)


class Mixed(C.Structure):
    """gmapdp_mixed (include/gmapdp.h): the drop-in's one-round-trip dispatcher batch."""
    _fields_ = [("singles", C.c_void_p), ("nsingle", C.c_int), ("ends", C.c_void_p), ("nend", C.c_int),
                ("genomes", C.c_void_p), ("ngenome", C.c_int), ("splice_probs", C.c_void_p), ("nprobs", C.c_size_t),
                ("results", C.c_void_p), ("genome_results", C.c_void_p), ("pairs", C.c_void_p),
                ("pair_capacity", C.c_size_t), ("searches", C.c_void_p), ("nsearch", C.c_int),
                ("search_results", C.c_void_p), ("candidates", C.c_void_p), ("candidate_capacity", C.c_size_t),
                ("candidates_needed", C.c_size_t), ("finishes", C.c_void_p), ("nfinish", C.c_int),
                ("finish_candidates", C.c_void_p), ("finish_probs", C.c_void_p), ("nfinish_candidates", C.c_size_t),
                ("finish_results", C.c_void_p), ("finish_pairs", C.c_void_p), ("finish_pair_capacity", C.c_size_t),
                ("known_sites", C.c_void_p), ("nknown", C.c_size_t), ("wholes", C.c_void_p), ("nwhole", C.c_int),
                ("whole_results", C.c_void_p), ("whole_pairs", C.c_void_p), ("whole_pair_capacity", C.c_size_t)]


_lib = None


def load_library(path=LIB_PATH):
    """Load libgmapdp.so; raises GmapdpError if the HIP extension is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise GmapdpError("libgmapdp.so not built (%s); run __graft_entry__.build()" % path)
    lib = C.CDLL(path)
    P = C.POINTER
    sig = {
        "gmapdp_create": (C.c_int, [P(C.c_void_p), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
        "gmapdp_destroy": (None, [C.c_void_p]),
        "gmapdp_create_ex": (C.c_int, [P(C.c_void_p), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
        "gmapdp_share_genome": (C.c_int, [C.c_void_p, C.c_void_p]),
        "gmapdp_dgenome_create": (C.c_int, [C.c_int, C.c_void_p, C.c_size_t, C.c_uint64, P(C.c_void_p)]),
        "gmapdp_dgenome_destroy": (None, [C.c_void_p]),
        "gmapdp_use_dgenome": (C.c_int, [C.c_void_p, C.c_void_p]),
        "gmapdp_reserve": (C.c_int, [C.c_void_p, C.c_size_t, C.c_int]),
        "gmapdp_genome_words": (C.c_size_t, [C.c_uint64]),
        "gmapdp_debug_stage2_scratch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
        "gmapdp_stage2_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_char_p, C.c_char_p, C.c_size_t,
                                          C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                          C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
        "gmapdp_pack_genome": (C.c_int, [C.c_char_p, C.c_uint64, C.c_void_p]),
        "gmapdp_set_genome": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint64]),
        "gmapdp_single_gap_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t,
                                              C.c_void_p, C.c_void_p, C.c_size_t]),
        "gmapdp_single_pair_capacity": (C.c_size_t, [C.c_void_p, C.c_int]),
        "gmapdp_end_gap_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t,
                                           C.c_void_p, C.c_void_p, C.c_size_t]),
        "gmapdp_end_pair_capacity": (C.c_size_t, [C.c_void_p, C.c_int]),
        "gmapdp_plan_create": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                                         P(C.c_void_p)]),
        "gmapdp_plan_single": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, P(C.c_void_p)]),
        "gmapdp_plan_pair_capacity": (C.c_size_t, [C.c_void_p]),
        "gmapdp_plan_gpu_problems": (C.c_int, [C.c_void_p]),
        "gmapdp_plan_dev_index": (C.c_int, [C.c_void_p, C.c_int]),
        "gmapdp_plan_nlaunches": (C.c_int, [C.c_void_p]),
        "gmapdp_plan_run": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p]),
        "gmapdp_plan_destroy": (None, [C.c_void_p]),
        "gmapdp_plan_launch_info": (C.c_int, [C.c_void_p, C.c_int, P(C.c_int), P(C.c_int), P(C.c_int),
                                              P(C.c_size_t)]),
        "gmapdp_plan_launch_members": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
        "gmapdp_plan_launch_is_tail": (C.c_int, [C.c_void_p, C.c_int]),
        "gmapdp_plan_launch_stream": (C.c_int, [C.c_void_p, C.c_int]),
        "gmapdp_plan_run_launch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_void_p, C.c_void_p]),
        "gmapdp_plan_run_launch_kernel": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                                    C.c_void_p, C.c_void_p, C.c_void_p]),
        "gmapdp_stream": (C.c_void_p, [C.c_void_p]),
        "gmapdp_genome_gap_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                              C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                              C.c_size_t]),
        "gmapdp_genome_pair_capacity": (C.c_size_t, [C.c_void_p, C.c_int]),
        "gmapdp_genome_gap_batch_known": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                                    C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                                    C.c_void_p, C.c_void_p, C.c_size_t]),
        "gmapdp_genome_known_bytes": (C.c_size_t, [C.c_void_p]),
        "gmapdp_dynprog_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                           C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_size_t]),
        "gmapdp_cdna_gap_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t,
                                            C.c_void_p, C.c_void_p, C.c_size_t]),
        "gmapdp_cdna_pair_capacity": (C.c_size_t, [C.c_void_p, C.c_int]),
        "gmapdp_end_splicejunction_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                                      C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                                      C.c_size_t]),
        "gmapdp_sj_pair_capacity": (C.c_size_t, [C.c_void_p, C.c_int]),
        "gmapdp_oligo_mappings_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_size_t,
                                                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                                  C.c_void_p, C.c_size_t]),
        "gmapdp_oligo_positions_capacity": (C.c_size_t, [C.c_void_p, C.c_int]),
        "gmapdp_oligo_diagonal_capacity": (C.c_size_t, [C.c_void_p, C.c_int]),
        "gmapdp_oligo_plan_create": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_size_t,
                                               P(C.c_void_p)]),
        "gmapdp_oligo_plan_positions_capacity": (C.c_size_t, [C.c_void_p]),
        "gmapdp_oligo_plan_diagonal_capacity": (C.c_size_t, [C.c_void_p]),
        "gmapdp_oligo_plan_nlaunches": (C.c_int, [C.c_void_p]),
        "gmapdp_oligo_plan_run": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_void_p]),
        "gmapdp_oligo_plan_destroy": (None, [C.c_void_p]),
        "gmapdp_stage2_plan_create": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t,
                                                P(C.c_void_p)]),
        "gmapdp_stage2_plan_run": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                             C.c_void_p]),
        "gmapdp_stage2_plan_outputs": (C.c_int, [C.c_void_p, P(C.c_void_p), P(C.c_void_p), P(C.c_void_p),
                                                 P(C.c_size_t)]),
        "gmapdp_stage2_plan_fetch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                               C.c_size_t, C.c_void_p, C.c_size_t, P(C.c_size_t), P(C.c_size_t)]),
        "gmapdp_stage2_plan_seeding_classes": (C.c_int, [C.c_void_p, P(C.c_int), P(C.c_int)]),
        "gmapdp_stage2_plan_seeding_results": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
        "gmapdp_stage2_plan_destroy": (None, [C.c_void_p]),
        "gmapdp_genome_prob_entries": (C.c_size_t, [C.c_void_p, C.c_int]),
        "gmapdp_genome_splice_sites": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t]),
        "gmapdp_plan_create_all": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                                             C.c_int, C.c_void_p, C.c_void_p, P(C.c_void_p)]),
        "gmapdp_plan_bind_genome": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
        "gmapdp_plan_genome_gpu_problems": (C.c_int, [C.c_void_p]),
        "gmapdp_plan_genome_dev_index": (C.c_int, [C.c_void_p, C.c_int]),
        "gmapdp_plan_launch_kind": (C.c_int, [C.c_void_p, C.c_int]),
        "gmapdp_compute_bands": (None, [P(C.c_int), P(C.c_int), C.c_int, C.c_int, C.c_int, C.c_int]),
        "gmapdp_last_error": (C.c_char_p, [C.c_void_p]),
        "gmapdp_microexon_search": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_char_p, C.c_char_p, C.c_size_t,
                                              C.c_void_p, C.c_void_p, C.c_size_t, P(C.c_size_t)]),
        "gmapdp_microexon_finish": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_char_p, C.c_char_p, C.c_size_t,
                                              C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                              C.c_size_t]),
        "gmapdp_microexon_pair_capacity": (C.c_size_t, [C.c_void_p, C.c_int]),
        "gmapdp_mixed_batch": (C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p, C.c_size_t, P(Mixed)]),
        "gmapdp_maxent_available": (C.c_int, [C.c_char_p, C.c_size_t]),
        "gmapdp_plan_bind_genome_maxent": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
        "gmapdp_plan_compact_bound": (C.c_size_t, [C.c_void_p]),
        "gmapdp_plan_compact_pairs": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                C.c_void_p, C.c_void_p]),
        "gmapdp_expand_pairs": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_int]),
        "gmapdp_stage2_plan_compact_bound": (C.c_size_t, [C.c_void_p, P(C.c_size_t)]),
        "gmapdp_stage2_plan_compact_pairs": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
        "gmapdp_expand_path_pairs": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int]),
        "gmapdp_maxent_sites": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
        "gmapdp_microexon_plan_create": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                                   C.c_size_t, P(C.c_void_p)]),
        "gmapdp_microexon_plan_candidates": (C.c_size_t, [C.c_void_p]),
        "gmapdp_microexon_plan_pair_capacity": (C.c_size_t, [C.c_void_p]),
        "gmapdp_microexon_plan_device_candidates": (C.c_void_p, [C.c_void_p]),
        "gmapdp_microexon_plan_run": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
        "gmapdp_microexon_plan_destroy": (None, [C.c_void_p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


_HIP = None


def _hip():
    """The HIP runtime (device buffers for the plan APIs' caller-owned device arguments)."""
    global _HIP
    if _HIP is None:
        h = C.CDLL("libamdhip64.so")
        h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        h.hipFree.argtypes = [C.c_void_p]
        _HIP = h
    return _HIP


def exported_symbols():
    """Names of the C ABI functions declared in include/gmapdp.h."""
    hdr = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "gmapdp.h")
    import re
    txt = open(hdr).read()
    return sorted(set(re.findall(r"\b(gmapdp_[a-z_0-9]+)\s*\(", txt)))


def pack_genome(seq: bytes) -> np.ndarray:
    """Compress_create_blocks_comp-format packing (compress-write.c:754)."""
    lib = load_library()
    n = lib.gmapdp_genome_words(len(seq))
    out = np.zeros(n, dtype=np.uint32)
    rc = lib.gmapdp_pack_genome(seq, len(seq), out.ctypes.data)
    if rc:
        raise GmapdpError("gmapdp_pack_genome failed: %d" % rc)
    return out


def build_genome_batch(calls):
    """calls: dicts with the Dynprog_genome_gap arguments (q, quc, rlength, glengthL, glengthR, roffset,
    goffsetL, rev_goffsetR, chroffset, chrhigh, cdna_direction, flags, genestrand, extraband, defect_rate,
    maxpeelback, dynprogindex).  Returns (problems, qbuf, qucbuf, nprob_entries); problem i's splice
    probabilities go at [prob_offset, +glengthL+glengthR) of a double arena."""
    calls = list(calls)
    probs = np.zeros(len(calls), dtype=GENOME_PROBLEM_DTYPE)
    qparts, qucparts, off, poff = [], [], 0, 0
    for i, p in enumerate(calls):
        probs[i]["qoff"] = off
        for k in ("rlength", "glengthL", "glengthR", "roffset", "goffsetL", "rev_goffsetR", "chroffset", "chrhigh",
                  "flags", "cdna_direction", "genestrand", "extraband", "maxpeelback", "dynprogindex",
                  "defect_rate"):
            probs[i][k] = p[k]
        if p.get("simd"):
            probs[i]["flags"] |= SIMD
        probs[i]["prob_offset"] = poff
        poff += max(0, p["glengthL"]) + max(0, p["glengthR"])
        qparts.append(p["q"])
        qucparts.append(p["quc"])
        off += len(p["q"])
    return probs, (b"".join(qparts) or b"\0"), (b"".join(qucparts) or b"\0"), poff


def genome_splice_sites(probs):
    """(positions uint64, models uint8) of every splice-probability entry: the Maxent_hr_*_prob
    calls (model 0 donor, 1 acceptor, 2 antidonor, 3 antiacceptor) whose values the engine reads."""
    lib = load_library()
    n = len(probs)
    m = lib.gmapdp_genome_prob_entries(probs.ctypes.data, n)
    pos = np.zeros(max(m, 1), dtype=np.uint64)
    mod = np.zeros(max(m, 1), dtype=np.uint8)
    rc = lib.gmapdp_genome_splice_sites(probs.ctypes.data, n, pos.ctypes.data, mod.ctypes.data, m)
    if rc:
        raise GmapdpError("gmapdp_genome_splice_sites failed: %d" % rc)
    return pos[:m], mod[:m]


class Engine:
    """One Dynprog engine context on one GPU (mirrors a GMAP worker's Dynprog_T)."""

    def __init__(self, device=0, mode=0, user_open=0, user_extend=0, user_dynprog_p=False, flags=0):
        self.lib = load_library()
        h = C.c_void_p()
        rc = self.lib.gmapdp_create_ex(C.byref(h), device, mode, user_open, user_extend, int(bool(user_dynprog_p)),
                                       flags)
        if rc:
            raise GmapdpError("gmapdp_create failed (%d): no usable HIP device %d?" % (rc, device))
        self.h = h
        self.genome_length = 0

    def close(self):
        if self.h:
            self.lib.gmapdp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc:
            raise GmapdpError("%s failed (%d): %s" % (what, rc, self.lib.gmapdp_last_error(self.h).decode()))

    def share_genome(self, owner):
        """Use `owner`'s HBM genome (gmapdp_share_genome); `owner` must stay open meanwhile."""
        self._check(self.lib.gmapdp_share_genome(self.h, owner.h), "gmapdp_share_genome")
        self.genome_length = owner.genome_length

    def set_genome(self, seq: bytes = None, blocks: np.ndarray = None, length: int = None):
        if blocks is None:
            blocks = pack_genome(seq)
            length = len(seq)
        blocks = np.ascontiguousarray(blocks, dtype=np.uint32)
        self._check(self.lib.gmapdp_set_genome(self.h, blocks.ctypes.data, blocks.size, length), "gmapdp_set_genome")
        self.genome_length = length

    # -- batched Dynprog_single_gap ------------------------------------------
    @staticmethod
    def build_single_batch(calls):
        """calls: iterable of dicts with the Dynprog_single_gap arguments
        (q, quc, rlength, glength, roffset, goffset, chroffset, chrhigh, watsonp, genestrand,
        jump_late_p, extraband, widebandp, defect_rate, dynprogindex)."""
        calls = list(calls)
        probs = np.zeros(len(calls), dtype=PROBLEM_DTYPE)
        qparts, qucparts, off = [], [], 0
        for i, p in enumerate(calls):
            q, quc = p["q"], p["quc"]
            probs[i]["qoff"] = off
            probs[i]["rlength"] = p["rlength"]
            probs[i]["glength"] = p["glength"]
            probs[i]["roffset"] = p["roffset"]
            probs[i]["goffset"] = p["goffset"]
            probs[i]["chroffset"] = p["chroffset"]
            probs[i]["chrhigh"] = p["chrhigh"]
            probs[i]["flags"] = ((WATSON if p["watsonp"] else 0) | (JUMP_LATE if p["jump_late_p"] else 0) |
                                 (WIDEBAND if p["widebandp"] else 0) | (SIMD if p.get("simd") else 0))
            probs[i]["genestrand"] = p["genestrand"]
            probs[i]["extraband"] = p["extraband"]
            probs[i]["defect_rate"] = p["defect_rate"]
            probs[i]["dynprogindex"] = p["dynprogindex"]
            qparts.append(q)
            qucparts.append(quc)
            off += len(q)
        qbuf = b"".join(qparts) or b"\0"
        qucbuf = b"".join(qucparts) or b"\0"
        return probs, qbuf, qucbuf

    def single_gap_batch_raw(self, probs, qbuf, qucbuf):
        n = len(probs)
        results = np.zeros(n, dtype=RESULT_DTYPE)
        cap = self.lib.gmapdp_single_pair_capacity(probs.ctypes.data, n)
        pairs = np.zeros(max(cap, 1), dtype=PAIR_DTYPE)
        rc = self.lib.gmapdp_single_gap_batch(self.h, probs.ctypes.data, n, qbuf, qucbuf, len(qbuf),
                                              results.ctypes.data, pairs.ctypes.data, cap)
        self._check(rc, "gmapdp_single_gap_batch")
        return results, pairs

    def single_gap_batch(self, calls):
        """Returns, per call, ((dynprogindex, traceback_score, nmatches, nmismatches, nopens, nindels),
        pairs-or-None) with pairs in the reference's list order as tuples
        (querypos, genomepos, queryjump, genomejump, dynprogindex, cdna, comp, genome, genomealt, gapp)."""
        calls = list(calls)
        probs, qbuf, qucbuf = self.build_single_batch(calls)
        results, pairs = self.single_gap_batch_raw(probs, qbuf, qucbuf)
        return decode_results(results, pairs, [p["dynprogindex"] for p in calls])


    # -- batched Dynprog_end5_gap / Dynprog_end3_gap ---------------------------
    @staticmethod
    def build_end_batch(calls):
        """calls: dicts with the Dynprog_end{5,3}_gap arguments (end3p, q, quc, rlength, glength, roffset,
        goffset, chroffset, chrhigh, watsonp, genestrand, jump_late_p, extraband, defect_rate, endalign,
        require_pos_score_p, dynprogindex); q/quc is the query slice the reference reads (end5: its
        rev pointer is the slice's last character)."""
        calls = list(calls)
        probs = np.zeros(len(calls), dtype=END_PROBLEM_DTYPE)
        qparts, qucparts, off = [], [], 0
        for i, p in enumerate(calls):
            q, quc = p["q"], p["quc"]
            probs[i]["qoff"] = off
            for k in ("rlength", "glength", "roffset", "goffset", "chroffset", "chrhigh", "genestrand",
                      "end3p", "endalign", "require_pos_score_p", "dynprogindex", "defect_rate"):
                probs[i][k] = p[k]
            probs[i]["extraband"] = p["extraband"]
            probs[i]["flags"] = ((WATSON if p["watsonp"] else 0) | (JUMP_LATE if p["jump_late_p"] else 0) |
                                 (SIMD if p.get("simd") else 0))
            qparts.append(q)
            qucparts.append(quc)
            off += len(q)
        return probs, (b"".join(qparts) or b"\0"), (b"".join(qucparts) or b"\0")

    def end_gap_batch(self, calls):
        calls = list(calls)
        probs, qbuf, qucbuf = self.build_end_batch(calls)
        n = len(probs)
        results = np.zeros(n, dtype=RESULT_DTYPE)
        cap = self.lib.gmapdp_end_pair_capacity(probs.ctypes.data, n)
        pairs = np.zeros(max(cap, 1), dtype=PAIR_DTYPE)
        rc = self.lib.gmapdp_end_gap_batch(self.h, probs.ctypes.data, n, qbuf, qucbuf, len(qbuf),
                                           results.ctypes.data, pairs.ctypes.data, cap)
        self._check(rc, "gmapdp_end_gap_batch")
        return decode_results(results, pairs, [p["dynprogindex"] for p in calls])


    # -- batched Dynprog_end5/3_splicejunction --------------------------------
    @staticmethod
    def build_sj_batch(calls):
        """calls: dicts with the Dynprog_end{5,3}_splicejunction arguments (end3p, q, quc, j, rlength, glength,
        roffset, goffset_anchor, goffset_far, contlength, genestrand, jump_late_p, extraband, defect_rate,
        dynprogindex); q/quc is the query slice and j the junction string the reference reads (end5: both
        rev pointers are the slices' last characters)."""
        calls = list(calls)
        probs = np.zeros(len(calls), dtype=SJ_PROBLEM_DTYPE)
        qparts, qucparts, jparts, off, joff = [], [], [], 0, 0
        for i, p in enumerate(calls):
            probs[i]["qoff"] = off
            probs[i]["joff"] = joff
            for k in ("rlength", "glength", "roffset", "goffset_anchor", "goffset_far", "contlength", "genestrand",
                      "end3p", "dynprogindex", "defect_rate"):
                probs[i][k] = p[k]
            probs[i]["extraband"] = p["extraband"]
            probs[i]["flags"] = (JUMP_LATE if p["jump_late_p"] else 0) | (SIMD if p.get("simd") else 0)
            qparts.append(p["q"])
            qucparts.append(p["quc"])
            jparts.append(p["j"])
            off += len(p["q"])
            joff += len(p["j"])
        return probs, (b"".join(qparts) or b"\0"), (b"".join(qucparts) or b"\0"), (b"".join(jparts) or b"\0")

    def end_splicejunction_batch(self, calls):
        """Per call ((dynprogindex, traceback_score, missscore, nmatches, nmismatches, nopens, nindels,
        known_index), pairs-or-None), as the oracle's end_splicejunction."""
        calls = list(calls)
        probs, qbuf, qucbuf, jbuf = self.build_sj_batch(calls)
        n = len(probs)
        results = np.zeros(n, dtype=SJ_RESULT_DTYPE)
        cap = self.lib.gmapdp_sj_pair_capacity(probs.ctypes.data, n)
        pairs = np.zeros(max(cap, 1), dtype=PAIR_DTYPE)
        rc = self.lib.gmapdp_end_splicejunction_batch(self.h, probs.ctypes.data, n, qbuf, qucbuf, len(qbuf), jbuf,
                                                      len(jbuf), results.ctypes.data, pairs.ctypes.data, cap)
        self._check(rc, "gmapdp_end_splicejunction_batch")
        out = []
        for i, res in enumerate(results):
            scal = tuple(int(res[k]) for k in ("dynprogindex", "traceback_score", "missscore", "nmatches",
                                                "nmismatches", "nopens", "nindels", "known_index"))
            n_ = int(res["npairs"])
            out.append((scal, None if n_ == 0 else
                        decode_pairs(pairs, int(res["pair_offset"]), n_, calls[i]["dynprogindex"])))
        return out

    # -- device MaxEnt (Maxent_hr_*_prob, maxent_hr.c:27357-27652) ------------------------------------
    def maxent_sites(self, positions, models, chroffsets):
        """Maxent_hr_<model>_prob(splice_pos, chroffset) per entry on the device (model GMAPDP_MAXENT_*)."""
        pos = np.ascontiguousarray(positions, dtype=np.uint64)
        mod = np.ascontiguousarray(models, dtype=np.uint8)
        chro = np.ascontiguousarray(np.broadcast_to(np.asarray(chroffsets, dtype=np.uint64), pos.shape))
        out = np.zeros(len(pos), dtype=np.float64)
        self._check(self.lib.gmapdp_maxent_sites(self.h, pos.ctypes.data, mod.ctypes.data, chro.ctypes.data, len(pos),
                                                 out.ctypes.data), "gmapdp_maxent_sites")
        return out

    # -- batched Dynprog_genome_gap -------------------------------------------
    def genome_gap_batch_raw(self, probs, qbuf, qucbuf, splice_probs):
        """splice_probs: the probability arena, or DEVICE (the engine's device MaxEnt: a NULL arena)."""
        n = len(probs)
        results = np.zeros(n, dtype=GENOME_RESULT_DTYPE)
        cap = self.lib.gmapdp_genome_pair_capacity(probs.ctypes.data, n)
        pairs = np.zeros(max(cap, 1), dtype=PAIR_DTYPE)
        if isinstance(splice_probs, str) and splice_probs == DEVICE:
            sp_ptr, nsp = None, 0
        else:
            sp = np.ascontiguousarray(splice_probs, dtype=np.float64)
            if sp.size == 0:
                sp = np.zeros(1)
            sp_ptr, nsp = sp.ctypes.data, len(splice_probs)
        rc = self.lib.gmapdp_genome_gap_batch(self.h, probs.ctypes.data, n, qbuf, qucbuf, len(qbuf), sp_ptr,
                                              nsp, results.ctypes.data, pairs.ctypes.data, cap)
        self._check(rc, "gmapdp_genome_gap_batch")
        return results, pairs

    def genome_gap_batch(self, calls, splice_probs):
        """splice_probs: per call (left_probs, right_probs) lists.  Returns per call
        ((dpi, score, nmatches, nmismatches, nopens, nindels, new_left, new_right, exonhead, introntype,
        left_prob, right_prob), pairs-or-None) in the oracle's format (the intron gap holder carries
        the queryjump)."""
        calls = list(calls)
        probs, qbuf, qucbuf, m = build_genome_batch(calls)
        if isinstance(splice_probs, str) and splice_probs == DEVICE:
            results, pairs = self.genome_gap_batch_raw(probs, qbuf, qucbuf, DEVICE)
            return decode_genome_results(results, pairs, [p["dynprogindex"] for p in calls])
        arena = np.zeros(max(m, 1))
        for i, (lp, rp) in enumerate(splice_probs):
            o = int(probs[i]["prob_offset"])
            arena[o:o + len(lp)] = lp
            arena[o + len(lp):o + len(lp) + len(rp)] = rp
        results, pairs = self.genome_gap_batch_raw(probs, qbuf, qucbuf, arena[:m])
        return decode_genome_results(results, pairs, [p["dynprogindex"] for p in calls])

    def genome_gap_batch_known(self, calls, splice_probs, known):
        """genome_gap_batch with known splice sites (GMAPDP_KNOWN_SITES): known[i] is call i's flag bytes
        in the include/gmapdp.h layout (bridge left, bridge right, simple left, simple right), or None."""
        calls = list(calls)
        probs, qbuf, qucbuf, m = build_genome_batch(calls)
        dev = isinstance(splice_probs, str) and splice_probs == DEVICE
        arena = np.zeros(max(m, 1))
        for i, (lp, rp) in enumerate([] if dev else splice_probs):
            o = int(probs[i]["prob_offset"])
            arena[o:o + len(lp)] = lp
            arena[o + len(lp):o + len(lp) + len(rp)] = rp
        kparts, ko = [], 0
        for i, k in enumerate(known):
            if k is None:
                continue
            probs[i]["flags"] |= KNOWN_SITES
            probs[i]["known_offset"] = ko
            kparts.append(bytes(k))
            ko += len(k)
        kb = np.frombuffer(b"".join(kparts) or b"\0", dtype=np.uint8).copy()
        n = len(probs)
        results = np.zeros(n, dtype=GENOME_RESULT_DTYPE)
        cap = self.lib.gmapdp_genome_pair_capacity(probs.ctypes.data, n)
        pairs = np.zeros(max(cap, 1), dtype=PAIR_DTYPE)
        sp = np.ascontiguousarray(arena[:max(m, 1)])
        rc = self.lib.gmapdp_genome_gap_batch_known(self.h, probs.ctypes.data, n, qbuf, qucbuf, len(qbuf),
                                                    None if dev else sp.ctypes.data, m, kb.ctypes.data, ko,
                                                    results.ctypes.data,
                                                    pairs.ctypes.data, cap)
        self._check(rc, "gmapdp_genome_gap_batch_known")
        return decode_genome_results(results, pairs, [p["dynprogindex"] for p in calls])

    # -- batched Dynprog_cdna_gap ---------------------------------------------
    @staticmethod
    def build_cdna_batch(calls):
        """calls: dicts with the Dynprog_cdna_gap arguments (q, quc, qposL, qposR, rlengthL, rlengthR, glength,
        roffsetL, rev_roffsetR, goffset, chroffset, chrhigh, watsonp, genestrand, jump_late_p, extraband,
        defect_rate, dynprogindex); rsequenceL = q + qposL, rev_rsequenceR = q + qposR."""
        calls = list(calls)
        probs = np.zeros(len(calls), dtype=CDNA_PROBLEM_DTYPE)
        qparts, qucparts, off = [], [], 0
        for i, p in enumerate(calls):
            probs[i]["qoffL"] = off + p["qposL"]
            probs[i]["qoffR"] = off + p["qposR"]
            for k in ("rlengthL", "rlengthR", "glength", "roffsetL", "rev_roffsetR", "goffset", "chroffset",
                      "chrhigh", "genestrand", "extraband", "dynprogindex", "defect_rate"):
                probs[i][k] = p[k]
            probs[i]["flags"] = ((WATSON if p["watsonp"] else 0) | (JUMP_LATE if p["jump_late_p"] else 0) |
                                 (SIMD if p.get("simd") else 0))
            qparts.append(p["q"])
            qucparts.append(p["quc"])
            off += len(p["q"])
        return probs, (b"".join(qparts) or b"\0"), (b"".join(qucparts) or b"\0")

    def cdna_gap_batch(self, calls):
        """Returns per call ((dynprogindex, traceback_score, incompletep), pairs-or-None) in the oracle's
        format (the gap holder carries the queryjump)."""
        calls = list(calls)
        probs, qbuf, qucbuf = self.build_cdna_batch(calls)
        n = len(probs)
        results = np.zeros(n, dtype=CDNA_RESULT_DTYPE)
        cap = self.lib.gmapdp_cdna_pair_capacity(probs.ctypes.data, n)
        pairs = np.zeros(max(cap, 1), dtype=PAIR_DTYPE)
        rc = self.lib.gmapdp_cdna_gap_batch(self.h, probs.ctypes.data, n, qbuf, qucbuf, len(qbuf),
                                            results.ctypes.data, pairs.ctypes.data, cap)
        self._check(rc, "gmapdp_cdna_gap_batch")
        out = []
        for i, res in enumerate(results):
            scal = (int(res["dynprogindex"]), int(res["traceback_score"]), int(res["incompletep"]))
            n_ = int(res["npairs"])
            lst = decode_pairs(pairs, int(res["pair_offset"]), n_, calls[i]["dynprogindex"]) if n_ else None
            if lst is not None and res["gap_index"] >= 0:
                g = int(res["gap_index"])
                lst[g] = (-1, -1, int(res["gap_queryjump"]), lst[g][3], 0, b" ", b" ", b" ", b" ", 1)
            out.append((scal, lst))
        return out

    # -- batched stage-2 seeding (Oligoindex_hr_tally + Oligoindex_get_mappings) --------------
    @staticmethod
    def build_oligo_batch(calls):
        """calls: dicts (quc, chrstart, chrend, chroffset, chrhigh, plusp, minor) -> (problems, qucbuf)."""
        calls = list(calls)
        probs = np.zeros(len(calls), dtype=OLIGO_PROBLEM_DTYPE)
        parts, off = [], 0
        for i, p in enumerate(calls):
            probs[i]["qoff"] = off
            probs[i]["querylength"] = len(p["quc"])
            for k in ("chrstart", "chrend", "chroffset", "chrhigh", "plusp", "minor"):
                probs[i][k] = int(p.get(k, 0))
            parts.append(p["quc"])
            off += len(p["quc"])
        return probs, (b"".join(parts) or b"\0")

    def oligo_mappings_batch_raw(self, probs, qucbuf):
        n = len(probs)
        results = np.zeros(n, dtype=OLIGO_RESULT_DTYPE)
        npos = np.zeros(max(len(qucbuf), 1), dtype=np.int32)
        maps = np.zeros(max(len(qucbuf), 1), dtype=np.int32)
        pc = self.lib.gmapdp_oligo_positions_capacity(probs.ctypes.data, n)
        dc = self.lib.gmapdp_oligo_diagonal_capacity(probs.ctypes.data, n)
        positions = np.zeros(max(pc, 1), dtype=np.uint32)
        diags = np.zeros(4 * max(dc, 1), dtype=np.int32)
        rc = self.lib.gmapdp_oligo_mappings_batch(self.h, probs.ctypes.data, n, qucbuf, len(qucbuf),
                                                  results.ctypes.data, npos.ctypes.data, maps.ctypes.data,
                                                  positions.ctypes.data, pc, diags.ctypes.data, dc)
        self._check(rc, "gmapdp_oligo_mappings_batch")
        return results, npos, maps, positions, diags

    def oligo_mappings_batch(self, calls):
        """Per call ((totalpositions, maxnconsecutive, oned_matrix_p, ndiagonals), npositions list,
        positions of every query position with hits concatenated in query order, diagonals as
        (diagonal, querystart, queryend, nconsecutive)) -- the oracle's format."""
        calls = list(calls)
        probs, qucbuf = self.build_oligo_batch(calls)
        results, npos, maps, positions, diags = self.oligo_mappings_batch_raw(probs, qucbuf)
        out = []
        for i, r in enumerate(results):
            o, n = int(probs[i]["qoff"]), int(probs[i]["querylength"])
            np_ = [int(x) for x in npos[o:o + n]]
            plist = []
            for q in range(n):
                if np_[q] > 0:
                    m = int(maps[o + q])
                    plist.extend(int(x) for x in positions[m:m + np_[q]])
            d0, nd = int(r["diag_offset"]), int(r["ndiagonals"])
            dg = [tuple(int(x) for x in diags[4 * (d0 + k):4 * (d0 + k) + 4]) for k in range(nd)]
            out.append(((int(r["totalpositions"]), int(r["maxnconsecutive"]), int(r["oned_matrix_p"]), nd),
                        np_, plist, dg))
        return out

    # -- batched Stage2_compute (seeding + chaining) -----------------------------------------------
    @staticmethod
    def build_stage2_batch(calls):
        """calls: dicts (q, quc, chrstart, chrend, chroffset, chrhigh, plusp, splicingp, maxintronlen)
        -> (problems, qbuf, qucbuf)."""
        calls = list(calls)
        probs = np.zeros(len(calls), dtype=STAGE2_PROBLEM_DTYPE)
        qs, qus, off = [], [], 0
        for i, p in enumerate(calls):
            probs[i]["qoff"] = off
            probs[i]["querylength"] = len(p["quc"])
            for k in ("chrstart", "chrend", "chroffset", "chrhigh", "plusp"):
                probs[i][k] = int(p.get(k, 0))
            probs[i]["splicingp"] = int(p.get("splicingp", 1))
            probs[i]["maxintronlen"] = int(p.get("maxintronlen", 500000))
            qs.append(p.get("q", p["quc"]))
            qus.append(p["quc"])
            off += len(p["quc"])
        return probs, (b"".join(qs) or b"\0"), (b"".join(qus) or b"\0")

    def stage2_batch_raw(self, probs, qbuf, qucbuf):
        n = len(probs)
        results = np.zeros(n, dtype=STAGE2_RESULT_DTYPE)
        pcap, qcap = 4 * n + 16, 2 * len(qucbuf) + 64
        while True:
            paths = np.zeros(pcap, dtype=PATH_DTYPE)
            pairs = np.zeros(qcap, dtype=PATH_PAIR_DTYPE)
            pn, qn = C.c_size_t(), C.c_size_t()
            rc = self.lib.gmapdp_stage2_batch(self.h, probs.ctypes.data, n, qbuf, qucbuf, len(qucbuf),
                                              results.ctypes.data, paths.ctypes.data, pcap, pairs.ctypes.data,
                                              qcap, C.byref(pn), C.byref(qn))
            if rc == -6:  # GMAPDP_ESPACE
                pcap, qcap = max(pcap, pn.value), max(qcap, qn.value)
                continue
            self._check(rc, "gmapdp_stage2_batch")
            return results, paths[:pn.value], pairs[:qn.value]

    def stage2_batch(self, calls):
        """Per call (number of results, [pair-key list per result]) -- the oracle's format (dpbind)."""
        calls = list(calls)
        probs, qbuf, qucbuf = self.build_stage2_batch(calls)
        results, paths, pairs = self.stage2_batch_raw(probs, qbuf, qucbuf)
        out = []
        for r in results:
            lists = []
            for k in range(int(r["nresults"])):
                pr = paths[int(r["path_offset"]) + k]
                o, m = int(pr["pair_offset"]), int(pr["npairs"])
                lst = []
                for x in pairs[o:o + m]:
                    gap = 1 if x["querypos"] == -1 and x["genomepos"] == -1 else 0
                    lst.append((int(x["querypos"]), int(x["genomepos"]), int(x["queryjump"]), int(x["genomejump"]), 0,
                                bytes(x["cdna"]) or b"\0", bytes(x["comp"]) or b"\0", bytes(x["genome"]) or b"\0",
                                bytes(x["genomealt"]) or b"\0", gap))
                lists.append(lst)
            out.append((int(r["nresults"]), lists))
        return out

    def stage2_plan_raw(self, probs, qbuf, qucbuf, run_qbuf=None, run_qucbuf=None, compact_out=None):
        """The device-resident Stage2_compute plan (bench.py's path): gmapdp_stage2_plan_create on
        (probs, qbuf, qucbuf) -- its sizing run, the measured re-layout, the 16-bit seeding class --,
        gmapdp_stage2_plan_run(what = 3) against device copies of the query arenas (run_qbuf /
        run_qucbuf when given: another query of the same layout), gmapdp_stage2_plan_fetch.  Returns
        (results, paths, pairs, (calls with 16-bit, with 32-bit seeding counters)).  compact_out (a dict):
        also the compact stream of the path pairs (gmapdp_stage2_plan_compact_pairs) expanded on the host
        (gmapdp_expand_path_pairs): compact_out["pairs"] (an arena like `pairs`), ["bytes"]."""
        lib, n = self.lib, len(probs)
        hip = _hip()
        plan = C.c_void_p()
        self._check(lib.gmapdp_stage2_plan_create(self.h, probs.ctypes.data, n, qbuf, qucbuf, len(qucbuf),
                                                  C.byref(plan)), "gmapdp_stage2_plan_create")
        bufs = []
        try:
            n16, n32 = C.c_int(), C.c_int()
            self._check(lib.gmapdp_stage2_plan_seeding_classes(plan, C.byref(n16), C.byref(n32)),
                        "gmapdp_stage2_plan_seeding_classes")

            def dbuf(nbytes, src=None):
                ptr = C.c_void_p()
                if hip.hipMalloc(C.byref(ptr), max(nbytes, 16)) != 0:
                    raise GmapdpError("hipMalloc(%d) failed" % nbytes)
                bufs.append(ptr)
                if src is not None and hip.hipMemcpy(ptr, src, nbytes, 1) != 0:  # hipMemcpyHostToDevice
                    raise GmapdpError("hipMemcpy failed")
                return ptr
            rq = qbuf if run_qbuf is None else run_qbuf
            rqu = qucbuf if run_qucbuf is None else run_qucbuf
            assert len(rq) == len(qbuf) and len(rqu) == len(qucbuf)
            d_q, d_quc = dbuf(len(rq), rq), dbuf(len(rqu), rqu)
            d_res = dbuf(n * STAGE2_RESULT_DTYPE.itemsize)
            self._check(lib.gmapdp_stage2_plan_run(self.h, plan, d_q, d_quc, d_res, 3, None), "gmapdp_stage2_plan_run")
            results = np.zeros(n, dtype=STAGE2_RESULT_DTYPE)
            pn, qn = C.c_size_t(), C.c_size_t()
            rc = lib.gmapdp_stage2_plan_fetch(self.h, plan, d_res, None, results.ctypes.data, None, 0, None, 0,
                                              C.byref(pn), C.byref(qn))
            if rc not in (0, -6):
                self._check(rc, "gmapdp_stage2_plan_fetch")
            paths = np.zeros(max(pn.value, 1), dtype=PATH_DTYPE)
            pairs = np.zeros(max(qn.value, 1), dtype=PATH_PAIR_DTYPE)
            self._check(lib.gmapdp_stage2_plan_fetch(self.h, plan, d_res, None, results.ctypes.data, paths.ctypes.data,
                                                     len(paths), pairs.ctypes.data, len(pairs), C.byref(pn),
                                                     C.byref(qn)), "gmapdp_stage2_plan_fetch")
            if compact_out is not None:
                pcap = C.c_size_t()
                bound = lib.gmapdp_stage2_plan_compact_bound(plan, C.byref(pcap))
                d_off, d_out = dbuf(8 * (pcap.value + 1)), dbuf(bound)
                self._check(lib.gmapdp_stage2_plan_compact_pairs(self.h, plan, d_out, d_off, None), "compact")
                if hip.hipDeviceSynchronize() != 0:
                    raise GmapdpError("hipDeviceSynchronize failed")
                offs = np.zeros(pn.value + 1, dtype=np.uint64)
                if hip.hipMemcpy(offs.ctypes.data, d_off, offs.nbytes, 2) != 0:  # hipMemcpyDeviceToHost
                    raise GmapdpError("hipMemcpy failed")
                stream = np.zeros(max(int(offs[-1]), 1), dtype=np.uint8)
                if hip.hipMemcpy(stream.ctypes.data, d_out, stream.nbytes, 2) != 0:
                    raise GmapdpError("hipMemcpy failed")
                compact_out["pairs"] = expand_path_pairs(stream, offs, paths[:pn.value], max(qn.value, 1))
                compact_out["bytes"] = int(offs[-1])
            return results, paths[:pn.value], pairs[:qn.value], (n16.value, n32.value)
        finally:
            for b in bufs:
                hip.hipFree(b)
            lib.gmapdp_stage2_plan_destroy(plan)

    # -- the drop-in's dispatcher batch (gmapdp_mixed_batch) ---------------------------------------
    def mixed_batch_raw(self, qbuf, qucbuf, singles=None, ends=None, genomes=None, splice_probs=None,
                        searches=None, finishes=None, finish_cands=None, finish_probs=None, finish_results=None,
                        candidate_capacity=None, wholes=None):
        """One gmapdp_mixed_batch call over one query arena (every section's qoff indexes qbuf).  Returns
        (return code, outputs: results, genome_results, pairs, search_results, candidates,
        candidates_needed, finish_results, finish_pairs) -- the caller checks the code (GMAPDP_ESPACE
        still fills the other sections)."""
        def arr(a, dt):
            return np.zeros(0, dtype=dt) if a is None else np.ascontiguousarray(a, dtype=dt)
        S, E = arr(singles, PROBLEM_DTYPE), arr(ends, END_PROBLEM_DTYPE)
        G = arr(genomes, GENOME_PROBLEM_DTYPE)
        XS, XF = arr(searches, MICROEXON_PROBLEM_DTYPE), arr(finishes, MICROEXON_PROBLEM_DTYPE)
        dev_sp = isinstance(splice_probs, str) and splice_probs == DEVICE
        dev_fp = isinstance(finish_probs, str) and finish_probs == DEVICE
        sp = arr(None if dev_sp else splice_probs, np.float64)
        fc, fp = arr(finish_cands, MICROEXON_CANDIDATE_DTYPE), arr(None if dev_fp else finish_probs, np.float64)
        XW = arr(wholes, MICROEXON_PROBLEM_DTYPE)
        fr = arr(finish_results, MICROEXON_RESULT_DTYPE).copy()
        lib = self.lib
        cap = (lib.gmapdp_single_pair_capacity(S.ctypes.data, len(S)) + lib.gmapdp_end_pair_capacity(E.ctypes.data, len(E))
               + lib.gmapdp_genome_pair_capacity(G.ctypes.data, len(G)))
        ccap = 16 * len(XS) + 4096 if candidate_capacity is None else candidate_capacity
        out = dict(results=np.zeros(max(1, len(S) + len(E)), dtype=RESULT_DTYPE),
                   genome_results=np.zeros(max(1, len(G)), dtype=GENOME_RESULT_DTYPE),
                   pairs=np.zeros(max(1, cap), dtype=PAIR_DTYPE),
                   search_results=np.zeros(max(1, len(XS)), dtype=MICROEXON_RESULT_DTYPE),
                   candidates=np.zeros(max(1, ccap), dtype=MICROEXON_CANDIDATE_DTYPE), finish_results=fr,
                   finish_pairs=np.zeros(max(1, lib.gmapdp_microexon_pair_capacity(XF.ctypes.data, len(XF))),
                                         dtype=PAIR_DTYPE),
                   whole_results=np.zeros(max(1, len(XW)), dtype=MICROEXON_RESULT_DTYPE),
                   whole_pairs=np.zeros(max(1, lib.gmapdp_microexon_pair_capacity(XW.ctypes.data, len(XW))),
                                        dtype=PAIR_DTYPE))
        m = Mixed(singles=S.ctypes.data, nsingle=len(S), ends=E.ctypes.data, nend=len(E), genomes=G.ctypes.data,
                  ngenome=len(G), splice_probs=None if dev_sp else sp.ctypes.data, nprobs=len(sp),
                  results=out["results"].ctypes.data,
                  genome_results=out["genome_results"].ctypes.data, pairs=out["pairs"].ctypes.data,
                  pair_capacity=cap, searches=XS.ctypes.data, nsearch=len(XS),
                  search_results=out["search_results"].ctypes.data, candidates=out["candidates"].ctypes.data,
                  candidate_capacity=ccap, finishes=XF.ctypes.data, nfinish=len(XF), finish_candidates=fc.ctypes.data,
                  finish_probs=None if dev_fp else fp.ctypes.data, nfinish_candidates=len(fc),
                  finish_results=fr.ctypes.data, finish_pairs=out["finish_pairs"].ctypes.data,
                  finish_pair_capacity=len(out["finish_pairs"]), wholes=XW.ctypes.data, nwhole=len(XW),
                  whole_results=out["whole_results"].ctypes.data, whole_pairs=out["whole_pairs"].ctypes.data,
                  whole_pair_capacity=len(out["whole_pairs"]))
        rc = lib.gmapdp_mixed_batch(self.h, qbuf, qucbuf, len(qbuf), C.byref(m))
        out["candidates_needed"] = int(m.candidates_needed)
        return rc, out


def decode_genome_results(results, pairs, dynprogindices):
    base = decode_results(results, pairs, dynprogindices)
    out = []
    for (scal, lst), res in zip(base, results):
        scal = scal + (int(res["new_leftgenomepos"]), int(res["new_rightgenomepos"]), int(res["exonhead"]),
                       int(res["introntype"]), float(res["left_prob"]), float(res["right_prob"]))
        if lst is not None and res["gap_index"] >= 0:
            g = int(res["gap_index"])
            lst[g] = (-1, -1, int(res["gap_queryjump"]), lst[g][3], 0, b" ", b" ", b" ", b" ", 1)
        out.append((scal, lst))
    return out


def _microexon_engine_methods():
    def build_microexon_batch(calls):
        """calls: dicts with the Dynprog_microexon_int arguments (q, quc: the query slice; rlength, roffset,
        goffsetL, rev_goffsetR, cdna_direction, chroffset, chrhigh, watsonp, genestrand, dynprogindex)."""
        calls = list(calls)
        probs = np.zeros(len(calls), dtype=MICROEXON_PROBLEM_DTYPE)
        off = 0
        for i, p in enumerate(calls):
            probs[i]["qoff"] = off
            for k in ("rlength", "roffset", "goffsetL", "rev_goffsetR", "cdna_direction", "chroffset", "chrhigh",
                      "watsonp", "genestrand", "dynprogindex"):
                probs[i][k] = p[k]
            off += len(p["q"])
        return probs, (b"".join(p["q"] for p in calls) or b"\0"), (b"".join(p["quc"] for p in calls) or b"\0")

    def microexon_search_raw(self, probs, qb, qub):
        n = len(probs)
        results = np.zeros(n, dtype=MICROEXON_RESULT_DTYPE)
        need = C.c_size_t(0)
        cands = np.zeros(max(1, 4 * n), dtype=MICROEXON_CANDIDATE_DTYPE)
        rc = self.lib.gmapdp_microexon_search(self.h, probs.ctypes.data, n, qb, qub, len(qb), results.ctypes.data,
                                              cands.ctypes.data, len(cands), C.byref(need))
        if rc == -6:
            cands = np.zeros(need.value, dtype=MICROEXON_CANDIDATE_DTYPE)
            rc = self.lib.gmapdp_microexon_search(self.h, probs.ctypes.data, n, qb, qub, len(qb),
                                                  results.ctypes.data, cands.ctypes.data, len(cands), C.byref(need))
        self._check(rc, "gmapdp_microexon_search")
        return results, cands[:need.value]

    def microexon_finish_raw(self, probs, qb, qub, cands, cand_probs, results):
        n = len(probs)
        cap = self.lib.gmapdp_microexon_pair_capacity(probs.ctypes.data, n)
        pairs = np.zeros(max(cap, 1), dtype=PAIR_DTYPE)
        dev = isinstance(cand_probs, str) and cand_probs == DEVICE
        cp = None if dev else np.ascontiguousarray(cand_probs, dtype=np.float64)
        if cp is not None and cp.size == 0:
            cp = np.zeros(2)
        res = results.copy()
        rc = self.lib.gmapdp_microexon_finish(self.h, probs.ctypes.data, n, qb, qub, len(qb), cands.ctypes.data,
                                              None if dev else cp.ctypes.data, len(cands), res.ctypes.data,
                                              pairs.ctypes.data, len(pairs))
        self._check(rc, "gmapdp_microexon_finish")
        return res, pairs

    def microexon_candidates(self, calls):
        """Per call the candidate tuples (cL, cR, candidate, middlelength, pos2, model2, pos3, model3) in the
        reference's loop order (None for cdna_direction 0), as the oracle lists them."""
        calls = list(calls)
        probs, qb, qub = build_microexon_batch(calls)
        results, cands = self.microexon_search_raw(probs, qb, qub)
        out = []
        for p, r in zip(calls, results):
            if p["cdna_direction"] == 0:
                out.append(None)
                continue
            o = int(r["cand_offset"])
            out.append([(int(c["cL"]), int(c["cR"]), int(c["candidate"]), int(c["middlelength"]), int(c["pos2"]),
                         int(c["model2"]), int(c["pos3"]), int(c["model3"]))
                        for c in cands[o:o + int(r["ncandidates"])]])
        return out

    def microexon_batch(self, calls, maxent):
        """Dynprog_microexon_int over a batch: search, the caller's MaxEnt (maxent(model, pos, chroffset)
        -> probability, e.g. the host's Maxent_hr_*_prob), finish.  Returns per call ((dynprogindex after,
        microintrontype), (bestprob2, bestprob3), pairs-or-None) in the oracle's format."""
        calls = list(calls)
        probs, qb, qub = build_microexon_batch(calls)
        results, cands = self.microexon_search_raw(probs, qb, qub)
        if isinstance(maxent, str) and maxent == DEVICE:
            res, pairs = self.microexon_finish_raw(probs, qb, qub, cands, DEVICE, results)
            return decode_microexon(calls, res, pairs)
        cp = np.zeros(2 * len(cands))
        for i, (p, r) in enumerate(zip(calls, results)):
            o = int(r["cand_offset"])
            for k in range(int(r["ncandidates"])):
                c = cands[o + k]
                cp[2 * (o + k)] = maxent(int(c["model2"]), int(c["pos2"]), p["chroffset"])
                cp[2 * (o + k) + 1] = maxent(int(c["model3"]), int(c["pos3"]), p["chroffset"])
        res, pairs = self.microexon_finish_raw(probs, qb, qub, cands, cp, results)
        return decode_microexon(calls, res, pairs)

    def microexon_whole_batch(self, calls):
        """Dynprog_microexon_int over a batch in ONE gmapdp_mixed_batch round trip (the whole-call section:
        search, device MaxEnt, choice); the same format as microexon_batch."""
        calls = list(calls)
        probs, qb, qub = build_microexon_batch(calls)
        rc, out = self.mixed_batch_raw(qb, qub, wholes=probs)
        self._check(rc, "gmapdp_mixed_batch (whole microexon calls)")
        return decode_microexon(calls, out["whole_results"], out["whole_pairs"])

    return dict(build_microexon_batch=staticmethod(build_microexon_batch), microexon_search_raw=microexon_search_raw,
                microexon_finish_raw=microexon_finish_raw, microexon_candidates=microexon_candidates,
                microexon_batch=microexon_batch, microexon_whole_batch=microexon_whole_batch)


def decode_microexon(calls, res, pairs):
    """Per call ((dynprogindex after, microintrontype), (bestprob2, bestprob3), pairs-or-None), the oracle's
    format, from gmapdp_microexon_result records and their pairs."""
    out = []
    for p, r in zip(calls, res):
        lst = None
        if r["npairs"] >= 0:
            lst = []
            for rec in pairs[int(r["pair_offset"]):int(r["pair_offset"]) + int(r["npairs"])]:
                if rec["querypos"] == -1 and rec["genomepos"] == -1:
                    lst.append((-1, -1, 0, int(rec["jump"]), 0, b" ", rec["comp"], b" ", b" ", 1))
                else:
                    lst.append((int(rec["querypos"]), int(rec["genomepos"]), 0, 0, p["dynprogindex"], rec["cdna"],
                                rec["comp"], rec["genome"], rec["genomealt"], 0))
        out.append(((int(r["dynprogindex"]), int(r["microintrontype"])),
                    (float(r["bestprob2"]), float(r["bestprob3"])), lst))
    return out


for _k, _v in _microexon_engine_methods().items():
    setattr(Engine, _k, _v)


def decode_results(results, pairs, dynprogindices):
    out = []
    for i, res in enumerate(results):
        scal = (int(res["dynprogindex"]), int(res["traceback_score"]), int(res["nmatches"]),
                int(res["nmismatches"]), int(res["nopens"]), int(res["nindels"]))
        n = int(res["npairs"])
        if n == 0:
            out.append((scal, None))
            continue
        out.append((scal, decode_pairs(pairs, int(res["pair_offset"]), n, dynprogindices[i])))
    return out


def decode_pairs(pairs, offset, n, dpi):
    """Pair records [offset, offset + n) as the oracle's Pair keys (gap holders: queryjump 0)."""
    lst = []
    for rec in pairs[offset:offset + n]:
        if rec["querypos"] == -1 and rec["genomepos"] == -1:
            lst.append((-1, -1, 0, int(rec["jump"]), 0, b" ", b" ", b" ", b" ", 1))
        else:
            lst.append((int(rec["querypos"]), int(rec["genomepos"]), 0, 0, dpi, rec["cdna"], rec["comp"],
                        rec["genome"], rec["genomealt"], 0))
    return lst


def expand_pairs(stream, offsets, npairs, pair_offsets, capacity, nthreads=0):
    """gmapdp_expand_pairs (host only): the compact pair stream back to gmapdp_pair records; a pair arena of
    `capacity` records with problem i's npairs[i] records at pair_offsets[i]."""
    lib = load_library()
    out = np.zeros(max(int(capacity), 1), dtype=PAIR_DTYPE)
    st = np.ascontiguousarray(stream, dtype=np.uint8)
    of = np.ascontiguousarray(offsets, dtype=np.uint64)
    npc = np.ascontiguousarray(npairs, dtype=np.int32)
    po = np.ascontiguousarray(pair_offsets, dtype=np.int64)
    rc = lib.gmapdp_expand_pairs(st.ctypes.data, of.ctypes.data, len(npc), npc.ctypes.data, po.ctypes.data,
                                 out.ctypes.data, int(nthreads))
    if rc != 0:
        raise GmapdpError("gmapdp_expand_pairs: the stream does not decode to the records (%d)" % rc)
    return out


def expand_path_pairs(stream, offsets, paths, capacity, nthreads=0):
    """gmapdp_expand_path_pairs (host only): a stage-2 plan's compact path-pair stream back to gmapdp_path_pair
    records; a pair arena of `capacity` records with each path's npairs at its pair_offset (`paths`: the
    plan's PATH_DTYPE records, one stream list each)."""
    lib = load_library()
    out = np.zeros(max(int(capacity), 1), dtype=PATH_PAIR_DTYPE)
    st = np.ascontiguousarray(stream, dtype=np.uint8)
    of = np.ascontiguousarray(offsets, dtype=np.uint64)
    pa = np.ascontiguousarray(paths, dtype=PATH_DTYPE)
    rc = lib.gmapdp_expand_path_pairs(st.ctypes.data, of.ctypes.data, len(pa), pa.ctypes.data, out.ctypes.data,
                                      int(nthreads))
    if rc != 0:
        raise GmapdpError("gmapdp_expand_path_pairs: the stream does not decode to the records (%d)" % rc)
    return out
