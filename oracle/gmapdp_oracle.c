/* oracle/gmapdp_oracle.c -- TEST INFRASTRUCTURE ONLY (see gmapdp_oracle.h).
 *
 * Plain-C restatement of the reference's nosimd Dynprog_* path.  Every
 * function names the reference code it restates (paths relative to
 * /root/reference/src).  Checked against the reference's own objects by
 * tests/test_oracle_vs_ref.py and against tests/golden/ vectors.
 */
#include <ctype.h>
#include <stdlib.h>
#include <string.h>

#include "gmapdp_oracle.h"

/* ---- constants (dynprog.h:44-119, dynprog.c:104, scores.h, comp.h) ---- */
enum { HIGHQ = 0, MEDQ = 1, LOWQ = 2, ENDQ = 3 };
#define FULLMATCH 3
#define HALFMATCH 1
#define AMBIGUOUS 3
#define MISMATCH_HIGHQ -3
#define MISMATCH_MEDQ -2
#define MISMATCH_LOWQ -1
#define MISMATCH_ENDQ -5
#define DEFECT_HIGHQ 0.003
#define DEFECT_MEDQ 0.014
#define SINGLE_OPEN_HIGHQ -8
#define SINGLE_OPEN_MEDQ -7
#define SINGLE_OPEN_LOWQ -6
#define SINGLE_EXTEND_HIGHQ -3
#define SINGLE_EXTEND_MEDQ -2
#define SINGLE_EXTEND_LOWQ -1
#define NEG_INFINITY_8 (-128)
#define NEG_INFINITY_32 (-32768)
#define VERT -2
#define HORIZ -1
#define DIAG 0
#define MATCH 1
#define MISMATCH -3
#define QOPEN -3
#define QINDEL -1
#define TOPEN -3
#define TINDEL -1
#define DYNPROG_MATCH_COMP '*'
#define AMBIGUOUS_COMP ':'
#define MISMATCH_COMP ' '
#define INDEL_COMP '-'
#define MICROINTRON_LENGTH 9 /* pairpool.c: genome skips >= this become a gap holder */
#define LAZY_INDEL 1         /* dynprog.c:1791 */

/* Mode_T (mode.h:5) */
enum { STANDARD, CMET_STRANDED, CMET_NONSTRANDED, ATOI_STRANDED, ATOI_NONSTRANDED, TTOC_STRANDED, TTOC_NONSTRANDED };

/* complement.h:31 COMPLEMENT_LC (IUPAC complement, case preserving) */
static const char complCode[129] =
  "???????????????????????????????? ??#$%&')(*+,-./0123456789:;>=<??TVGHEFCDIJMLKNOPQYSAABWXRZ]?[^_`tvghefcdijmlknopqysaabwxrz}|{~?";

static short pairdistance[4][128][128];
static unsigned char consistent[3][128][128];
static int use8p_size[4];
static int g_mode;
static int g_simd;  /* 1: the SIMD (AVX2) build's semantics, 0: nosimd */
static int g_user_open, g_user_extend, g_user_dynprog_p;
static void intron_score_setup (void);

static const char *g_genome = NULL;
static unsigned int g_genomelength = 0;

/* ---------------------------------------------------------------------------
 * Score tables: restates Dynprog_init / permute_cases / permute_cases_oneway
 * (dynprog.c:903-1197).  Note the reference's loop bounds ('z' exclusive for
 * the second character, 'Z' exclusive for the identity loop) are kept.
 * ------------------------------------------------------------------------- */
static int
stranded_mode (int mode) {
  return mode == STANDARD || mode == CMET_STRANDED || mode == ATOI_STRANDED || mode == TTOC_STRANDED;
}

static void
set_both (int a, int b, short score, int mode) {
  int la = tolower(a), lb = tolower(b), t;
  int pairs[4][2] = {{la, lb}, {la, b}, {a, lb}, {a, b}};
  int k;
  for (k = 0; k < 4; k++) {
    if (stranded_mode(mode)) {
      consistent[0][pairs[k][0]][pairs[k][1]] = 1;
    } else {
      consistent[1][pairs[k][0]][pairs[k][1]] = 1;
      consistent[2][pairs[k][0]][pairs[k][1]] = 1;
    }
  }
  for (k = 0; k < 4; k++) {
    if (stranded_mode(mode)) {
      consistent[0][pairs[k][1]][pairs[k][0]] = 1;
    } else {
      consistent[1][pairs[k][1]][pairs[k][0]] = 1;
      consistent[2][pairs[k][1]][pairs[k][0]] = 1;
    }
  }
  for (t = 0; t < 4; t++) {
    for (k = 0; k < 4; k++) pairdistance[t][pairs[k][0]][pairs[k][1]] = score;
    for (k = 0; k < 4; k++) pairdistance[t][pairs[k][1]][pairs[k][0]] = score;
  }
}

static void
set_oneway (int a, int b, short score, int genestrand) {
  int la = tolower(a), lb = tolower(b), t;
  consistent[genestrand][la][lb] = 1;
  consistent[genestrand][la][b] = 1;
  consistent[genestrand][a][lb] = 1;
  consistent[genestrand][a][b] = 1;
  for (t = 0; t < 4; t++) {
    pairdistance[t][la][lb] = score;
    pairdistance[t][la][b] = score;
    pairdistance[t][a][lb] = score;
    pairdistance[t][a][b] = score;
  }
}

int
orc_init (int mode, int user_open, int user_extend, int user_dynprog_p) {
  int c1, c2;
  static const struct { char a, b; short s; } exc[] = {
    {'U','T',FULLMATCH},
    {'R','A',HALFMATCH},{'R','G',HALFMATCH},{'Y','T',HALFMATCH},{'Y','C',HALFMATCH},
    {'W','A',HALFMATCH},{'W','T',HALFMATCH},{'S','G',HALFMATCH},{'S','C',HALFMATCH},
    {'M','A',HALFMATCH},{'M','C',HALFMATCH},{'K','G',HALFMATCH},{'K','T',HALFMATCH},
    {'H','A',AMBIGUOUS},{'H','T',AMBIGUOUS},{'H','C',AMBIGUOUS},
    {'B','G',AMBIGUOUS},{'B','C',AMBIGUOUS},{'B','T',AMBIGUOUS},
    {'V','G',AMBIGUOUS},{'V','A',AMBIGUOUS},{'V','C',AMBIGUOUS},
    {'D','G',AMBIGUOUS},{'D','A',AMBIGUOUS},{'D','T',AMBIGUOUS},
    {'N','T',AMBIGUOUS},{'N','C',AMBIGUOUS},{'N','A',AMBIGUOUS},{'N','G',AMBIGUOUS},
    {'X','T',AMBIGUOUS},{'X','C',AMBIGUOUS},{'X','A',AMBIGUOUS},{'X','G',AMBIGUOUS},
    {'N','N',AMBIGUOUS},{'X','X',AMBIGUOUS},
  };
  size_t k;

  memset(pairdistance, 0, sizeof(pairdistance));
  memset(consistent, 0, sizeof(consistent));
  intron_score_setup();
  g_mode = mode;
  g_user_open = user_open;
  g_user_extend = user_extend;
  g_user_dynprog_p = user_dynprog_p;

  /* dynprog.c:1022-1025: NEG_INFINITY_8 / mismatch - 1 (C integer division) */
  use8p_size[HIGHQ] = NEG_INFINITY_8 / MISMATCH_HIGHQ - 1;
  use8p_size[MEDQ] = NEG_INFINITY_8 / MISMATCH_MEDQ - 1;
  use8p_size[LOWQ] = NEG_INFINITY_8 / MISMATCH_LOWQ - 1;
  use8p_size[ENDQ] = NEG_INFINITY_8 / MISMATCH_ENDQ - 1;

  for (c1 = 'A'; c1 <= 'z'; c1++) {
    for (c2 = 'A'; c2 < 'z'; c2++) {
      pairdistance[HIGHQ][c1][c2] = MISMATCH_HIGHQ;
      pairdistance[MEDQ][c1][c2] = MISMATCH_MEDQ;
      pairdistance[LOWQ][c1][c2] = MISMATCH_LOWQ;
      pairdistance[ENDQ][c1][c2] = MISMATCH_ENDQ;
    }
  }
  for (c1 = 'A'; c1 < 'Z'; c1++) set_both(c1, c1, FULLMATCH, mode);
  for (k = 0; k < sizeof(exc) / sizeof(exc[0]); k++) set_both(exc[k].a, exc[k].b, exc[k].s, mode);

  switch (mode) {
  case STANDARD: break;
  case CMET_STRANDED: set_oneway('T', 'C', FULLMATCH, 0); break;
  case CMET_NONSTRANDED: set_oneway('T', 'C', FULLMATCH, 1); set_oneway('A', 'G', FULLMATCH, 2); break;
  case ATOI_STRANDED: set_oneway('G', 'A', FULLMATCH, 0); break;
  case ATOI_NONSTRANDED: set_oneway('G', 'A', FULLMATCH, 1); set_oneway('C', 'T', FULLMATCH, 2); break;
  case TTOC_STRANDED: set_oneway('C', 'T', FULLMATCH, 0); break;
  case TTOC_NONSTRANDED: set_oneway('C', 'T', FULLMATCH, 1); set_oneway('G', 'A', FULLMATCH, 2); break;
  default: return -1;
  }
  return 0;
}

/* Select the semantics the oracle restates: 0 the nosimd build, 1 the SIMD (AVX2) build
   (Dynprog_simd_8/16 for single gaps, the _upper/_lower triangles for end and genome gaps). */
int
orc_set_simd (int simd) {
  g_simd = simd ? 1 : 0;
  return 0;
}

int
orc_pairdistance (int mismatchtype, short *out) {
  memcpy(out, pairdistance[mismatchtype], sizeof(pairdistance[0]));
  return 0;
}

int
orc_consistent (int genestrand, unsigned char *out) {
  memcpy(out, consistent[genestrand], sizeof(consistent[0]));
  return 0;
}

int
orc_set_genome (const char *genome, unsigned int length) {
  g_genome = genome;
  g_genomelength = length;
  return 0;
}

/* The genome bytes orc_set_genome holds (stage2_oracle.c reads them as .genomecomp codes). */
const char *
orc_genome_seq (unsigned int *length) {
  *length = g_genomelength;
  return g_genome;
}

/* ---------------------------------------------------------------------------
 * Genome access: get_genomic_nt (dynprog_single.c:116, pairpool.c) and
 * Genome_get_segment_right/left (genome.c:11023/11079).  Univcoord_T is the
 * 32-bit gmap type, so positions wrap exactly as in the reference.
 * ------------------------------------------------------------------------- */
static char
get_genomic_nt (char *g_alt, int genomicpos, unsigned int chroffset, unsigned int chrhigh, int watsonp) {
  unsigned int pos;
  char c;
  if (watsonp) {
    pos = chroffset + (unsigned int) genomicpos;
    if (pos < chroffset || pos >= chrhigh) { *g_alt = '*'; return '*'; }
    c = g_genome[pos];
    *g_alt = c;
    return c;
  } else {
    pos = chrhigh - (unsigned int) genomicpos;
    if (pos < chroffset || pos >= chrhigh) { *g_alt = '*'; return '*'; }
    c = g_genome[pos];
    *g_alt = complCode[(int) c];
    return complCode[(int) c];
  }
}

static void
complement_inplace (char *s, unsigned int length) {
  unsigned int i, j;
  char t;
  if (length == 0) return;
  for (i = 0, j = length - 1; i < length / 2; i++, j--) {
    t = complCode[(int) s[i]];
    s[i] = complCode[(int) s[j]];
    s[j] = t;
  }
  if (i == j) s[i] = complCode[(int) s[i]];
}

int
orc_get_segment (int rightp, unsigned int pos, int length_in, unsigned int chrbound, int revcomp,
                 char *segment, char *segmentalt) {
  unsigned int length = (unsigned int) length_in, oob, i;
  if (length == 0) { segment[0] = segmentalt[0] = '\0'; return 0; }
  if (rightp) {
    unsigned int left = pos, chrhigh = chrbound;
    if (left >= chrhigh) {
      for (i = 0; i < length; i++) segment[i] = segmentalt[i] = '*';
      segment[length] = segmentalt[length] = '\0';
      return 0;
    } else if (left + length >= chrhigh) {
      oob = left + length - chrhigh;
      for (i = length - 1; i + oob >= length; i--) segment[i] = '*';
    } else {
      oob = 0;
    }
    for (i = 0; i < length - oob; i++) segment[i] = g_genome[left + i];
  } else {
    unsigned int right = pos, chroffset = chrbound;
    if (right < chroffset) {
      for (i = 0; i < length; i++) segment[i] = segmentalt[i] = '*';
      segment[length] = segmentalt[length] = '\0';
      return 0;
    } else if (right < chroffset + length) {
      oob = chroffset + length - right;
      for (i = 0; i < oob; i++) segment[i] = '*';
    } else {
      oob = 0;
    }
    for (i = 0; i < length - oob; i++) segment[oob + i] = g_genome[right - length + oob + i];
  }
  segment[length] = '\0';
  if (revcomp) complement_inplace(segment, length);
  memcpy(segmentalt, segment, length);
  segmentalt[length] = '\0';
  return 0;
}

/* ---------------------------------------------------------------------------
 * Pair emission: Pairpool_push / _push_gapholder / _add_queryskip /
 * _add_genomeskip (pairpool.c:180,375,981,1068).  Pairs are recorded in PUSH
 * order; the reference list is the reverse of push order (each push
 * prepends).
 * ------------------------------------------------------------------------- */
typedef struct {
  OrcPair *buf;
  int n, cap;
} PairSink;

static void
sink_push (PairSink *s, int querypos, int genomepos, char cdna, char comp, char genome, char genomealt,
           int dynprogindex) {
  OrcPair *p;
  if (querypos < 0 || genomepos < 0) return; /* pairpool.c:188-190 */
  if (s->n < s->cap) {
    p = &s->buf[s->n];
    p->querypos = querypos; p->genomepos = genomepos; p->queryjump = 0; p->genomejump = 0;
    p->dynprogindex = dynprogindex; p->cdna = cdna; p->comp = comp; p->genome = genome;
    p->genomealt = genomealt; p->gapp = 0;
  }
  s->n++;
}

static void
sink_gapholder (PairSink *s, int queryjump, int genomejump) {
  OrcPair *p;
  if (s->n < s->cap) {
    p = &s->buf[s->n];
    p->querypos = -1; p->genomepos = -1; p->queryjump = queryjump; p->genomejump = genomejump;
    p->dynprogindex = 0; p->cdna = ' '; p->comp = ' '; p->genome = ' '; p->genomealt = ' '; p->gapp = 1;
  }
  s->n++;
}

static void
add_queryskip (PairSink *s, int r, int c, int dist, const char *qseq, int queryoffset, int genomeoffset,
               int revp, int dpi) {
  int j, querycoord = r - 1, genomecoord = c - 1, step;
  if (revp) { querycoord = -querycoord; genomecoord = -genomecoord; step = +1; } else { step = -1; }
  for (j = 0; j < dist; j++) {
    sink_push(s, queryoffset + querycoord, genomeoffset + genomecoord, qseq[querycoord], INDEL_COMP, ' ', ' ', dpi);
    querycoord += step;
  }
}

static int
add_genomeskip (PairSink *s, int r, int c, int dist, int queryoffset, int genomeoffset, int revp,
                unsigned int chroffset, unsigned int chrhigh, int watsonp, int dpi) {
  int j, querycoord = r - 1, left = c - dist, right = c - 1, t, genomecoord, step;
  char c2, c2_alt;
  if (revp) { querycoord = -querycoord; t = left; left = -right; right = -t; step = +1; } else { step = -1; }
  if (dist >= MICROINTRON_LENGTH) {
    sink_gapholder(s, 0, dist);
    return 0;
  }
  genomecoord = revp ? left : right;
  for (j = 0; j < dist; j++) {
    c2 = get_genomic_nt(&c2_alt, genomeoffset + genomecoord, chroffset, chrhigh, watsonp);
    sink_push(s, queryoffset + querycoord, genomeoffset + genomecoord, ' ', INDEL_COMP, c2, c2_alt, dpi);
    genomecoord += step;
  }
  return 1;
}

/* ---------------------------------------------------------------------------
 * Dynprog_standard (dynprog.c:1268-1786): banded affine-gap fill, column-major
 * over genome position c, rows r in [c-uband, c+lband].  The three direction
 * planes start cleared to DIAG (Directions32_alloc, dynprog.c:488-501).
 * ------------------------------------------------------------------------- */
#define IDX(c, r) ((size_t) (c) * (size_t) (rlength + 1) + (size_t) (r))

static inline int
prefer (int a, int b, int late) { return late ? (a >= b) : (a > b); }

int
orc_standard_fill (const char *rsequence, const char *gsequence, const char *gsequence_alt,
                   int rlength, int glength, int mismatchtype, int open, int extend,
                   int lband, int uband, int jump_late_p, int revp, int saturation,
                   int upperp, int lowerp, int *matrix, signed char *dirs) {
  size_t plane = (size_t) (glength + 1) * (size_t) (rlength + 1);
  signed char *dnogap = dirs, *dE = dirs + plane, *dF = dirs + 2 * plane;
  int *r_gap, *nogap;
  int penalty, c_gap, last_nogap, prev_nogap, first_nogap = 0, score, pairscore;
  int r, c, rlo, rhigh, na1, na2, na2_alt;
  short (*pd)[128] = pairdistance[mismatchtype];

  memset(matrix, 0, plane * sizeof(int));
  memset(dirs, DIAG, 3 * plane);

  /* row 0 and column 0 (INFINITE_INITIAL_GAP_PENALTY branch) */
  penalty = open;
  for (c = 1; c <= uband && c <= glength; c++) {
    penalty += extend;
    matrix[IDX(c, 0)] = penalty;
    dE[IDX(c, 0)] = HORIZ;
    dnogap[IDX(c, 0)] = HORIZ;
  }
  penalty = open;
  for (r = 1; r <= lband && r <= rlength; r++) {
    penalty += extend;
    matrix[IDX(0, r)] = penalty;
    dF[IDX(0, r)] = VERT;
    dnogap[IDX(0, r)] = VERT;
  }

  r_gap = (int *) malloc((rlength + 1) * sizeof(int));
  nogap = (int *) malloc((rlength + 1) * sizeof(int));
  nogap[0] = 0;
  penalty = open;
  for (r = 1; r <= lband && r <= rlength; r++) {
    penalty += extend;
    r_gap[r] = NEG_INFINITY_32;
    nogap[r] = penalty;
  }
  for (; r <= rlength; r++) {
    r_gap[r] = NEG_INFINITY_32;
    nogap[r] = NEG_INFINITY_32;
  }

  penalty = open + extend;
  for (c = 1; c <= glength; c++) {
    na2 = (unsigned char) (revp ? gsequence[1 - c] : gsequence[c - 1]);
    na2_alt = (unsigned char) (revp ? gsequence_alt[1 - c] : gsequence_alt[c - 1]);

    c_gap = NEG_INFINITY_32;
    if (c == 1) {
      rlo = 1;
      prev_nogap = 0;
      last_nogap = NEG_INFINITY_32 - open + 1;
    } else if ((rlo = c - uband) < 1) {
      rlo = 1;
      prev_nogap = penalty;
      penalty += extend;
      last_nogap = penalty;
    } else if (rlo == 1) {
      prev_nogap = penalty;
      last_nogap = NEG_INFINITY_32;
    } else {
      prev_nogap = first_nogap;
      last_nogap = NEG_INFINITY_32;
    }
    if ((rhigh = c + lband) > rlength) rhigh = rlength;

    for (r = rlo; r <= rhigh; r++) {
      na1 = (unsigned char) (revp ? rsequence[1 - r] : rsequence[r - 1]);

      /* F: vertical gap (query skip), chained down the column */
      score = last_nogap + open;
      if (lowerp && prefer(c_gap, score, jump_late_p)) {
        c_gap += extend;
        dF[IDX(c, r)] = VERT;
      } else {
        c_gap = score + extend;
      }

      /* E: horizontal gap (genome skip), chained along the row */
      score = nogap[r] + open;
      if (upperp && prefer(r_gap[r], score, jump_late_p)) {
        r_gap[r] += extend;
        dE[IDX(c, r)] = HORIZ;
      } else {
        r_gap[r] = score + extend;
      }

      /* H */
      pairscore = pd[na1][na2];
      if ((score = pd[na1][na2_alt]) > pairscore) pairscore = score;
      last_nogap = prev_nogap + pairscore;
      if (upperp && prefer(r_gap[r], last_nogap, jump_late_p)) {
        last_nogap = r_gap[r];
        dnogap[IDX(c, r)] = HORIZ;
      }
      if (lowerp && prefer(c_gap, last_nogap, jump_late_p)) {
        last_nogap = c_gap;
        dnogap[IDX(c, r)] = VERT;
      }

      prev_nogap = nogap[r];
      matrix[IDX(c, r)] = nogap[r] = (last_nogap < saturation) ? saturation : last_nogap;
      if (r == rlo) first_nogap = last_nogap;
    }
  }

  free(r_gap);
  free(nogap);
  return 0;
}

/* ---------------------------------------------------------------------------
 * Dynprog_traceback_std (dynprog.c:1796-1948)
 * ------------------------------------------------------------------------- */
typedef struct {
  int score, nmatches, nmismatches, nopens, nindels;
} Tally;

/* mode 0: Dynprog_traceback_std.  Modes 1/2: Dynprog_traceback_{8,16}_upper / _lower
   (dynprog_simd.c:9319/9439, 9716/9836) over one triangle's planes mapped into this layout
   (upper: nogap DIAG/HORIZ + Egap; lower: nogap DIAG/VERT + the vertical chain in dF).  Their
   walk is this one; only the final skip differs: upper always ends with a genome skip of c
   (the reference asserts r == 0), lower with a query skip of r (it asserts c == 0).  The
   chains keep the c > 0 / r > 0 guards: without them the reference would index before its
   arrays, which only a path through a diagonal tie at saturation can reach. */
static void
traceback_mode (PairSink *s, Tally *t, const signed char *dirs, int rlength, int glength, int r, int c,
                const char *rsequence, const char *rsequenceuc, const char *gsequence,
                const char *gsequence_alt, int queryoffset, int genomeoffset, int revp,
                unsigned int chroffset, unsigned int chrhigh, int watsonp, int genestrand, int dpi, int mode) {
  size_t plane = (size_t) (glength + 1) * (size_t) (rlength + 1);
  const signed char *dnogap = dirs, *dE = dirs + plane, *dF = dirs + 2 * plane;
  int dist, querycoord, genomecoord;
  signed char dir;
  char c1, c1_uc, c2, c2_alt;

  while (r > 0 && c > 0) {
    if ((dir = dnogap[IDX(c, r)]) == HORIZ) {
      dist = 1;
      while (c > 0 && dE[IDX(c--, r)] != DIAG) dist++;
      if (add_genomeskip(s, r, c + dist, dist, queryoffset, genomeoffset, revp, chroffset, chrhigh,
                         watsonp, dpi)) {
        t->score += TOPEN + dist * TINDEL;
        t->nopens += 1;
        t->nindels += dist;
      }
    } else if (dir == VERT) {
      dist = 1;
      while (r > 0 && dF[IDX(c, r--)] != DIAG) dist++;
      add_queryskip(s, r + dist, c, dist, rsequence, queryoffset, genomeoffset, revp, dpi);
      t->score += QOPEN + dist * QINDEL;
      t->nopens += 1;
      t->nindels += dist;
    } else {
      querycoord = r - 1;
      genomecoord = c - 1;
      if (revp) { querycoord = -querycoord; genomecoord = -genomecoord; }
      c1 = rsequence[querycoord];
      c1_uc = rsequenceuc[querycoord];
      c2 = gsequence[genomecoord];
      c2_alt = gsequence_alt[genomecoord];
      if (c2 == '*') {
        /* not pushed past the end of the chromosome */
      } else if (c1_uc == c2 || c1_uc == c2_alt) {
        t->score += MATCH; t->nmatches += 1;
        sink_push(s, queryoffset + querycoord, genomeoffset + genomecoord, c1, DYNPROG_MATCH_COMP, c2, c2_alt, dpi);
      } else if (consistent[genestrand][(unsigned char) c1_uc][(unsigned char) c2] ||
                 consistent[genestrand][(unsigned char) c1_uc][(unsigned char) c2_alt]) {
        t->score += MATCH; t->nmatches += 1;
        sink_push(s, queryoffset + querycoord, genomeoffset + genomecoord, c1, AMBIGUOUS_COMP, c2, c2_alt, dpi);
      } else {
        t->score += MISMATCH; t->nmismatches += 1;
        sink_push(s, queryoffset + querycoord, genomeoffset + genomecoord, c1, MISMATCH_COMP, c2, c2_alt, dpi);
      }
      r--; c--;
    }
  }

  if ((mode == 1 && c == 0) || (mode == 2 && r == 0) || (r == 0 && c == 0)) {
    /* finished with a diagonal step */
  } else if (mode == 2 || (mode == 0 && c == 0)) {
    dist = r;
    add_queryskip(s, r, 0 + LAZY_INDEL, dist, rsequence, queryoffset, genomeoffset, revp, dpi);
    t->score += QOPEN + dist * QINDEL;
    t->nopens += 1;
    t->nindels += dist;
  } else {
    dist = c;
    if (add_genomeskip(s, 0 + LAZY_INDEL, c, dist, queryoffset, genomeoffset, revp, chroffset, chrhigh,
                       watsonp, dpi)) {
      t->score += TOPEN + dist * TINDEL;
      t->nopens += 1;
      t->nindels += dist;
    }
  }
}

static void
traceback_std (PairSink *s, Tally *t, const signed char *dirs, int rlength, int glength, int r, int c,
               const char *rsequence, const char *rsequenceuc, const char *gsequence,
               const char *gsequence_alt, int queryoffset, int genomeoffset, int revp,
               unsigned int chroffset, unsigned int chrhigh, int watsonp, int genestrand, int dpi) {
  traceback_mode(s, t, dirs, rlength, glength, r, c, rsequence, rsequenceuc, gsequence, gsequence_alt,
                 queryoffset, genomeoffset, revp, chroffset, chrhigh, watsonp, genestrand, dpi, 0);
}

/* Dynprog_compute_bands (dynprog.c:1247) */
static void
compute_bands (int *lband, int *uband, int rlength, int glength, int extraband, int widebandp) {
  if (!widebandp) { *lband = extraband; *uband = extraband; }
  else if (glength >= rlength) { *uband = glength - rlength + extraband; *lband = extraband; }
  else { *lband = rlength - glength + extraband; *uband = extraband; }
}

/* ---------------------------------------------------------------------------
 * Dynprog_single_gap (dynprog_single.c:429-676), nosimd build, homopolymerp
 * false (the default; dynprog_single.c:535 is out of scope).  Max lengths are
 * those of Dynprog_new with gmap.c's defaults (dynprog.c:602-627):
 * max_rlength 660, max_glength 2000.
 * ------------------------------------------------------------------------- */
#define ORC_MAX_RLENGTH 660
#define ORC_MAX_GLENGTH 2000

/* single_gap_simple (dynprog_single.c:346) */
static int
single_gap_simple (PairSink *s, Tally *t, const char *rsequence, const char *rsequenceuc, int rlength,
                   const char *gsequence, const char *gsequence_alt, int roffset, int goffset,
                   int genestrand, int dpi) {
  int r, q;
  char c1, c1_uc, c2, c2_alt;
  t->score = 0; t->nmatches = t->nmismatches = 0;
  for (r = 1; r <= rlength; r++) {
    q = r - 1;
    c1 = rsequence[q]; c1_uc = rsequenceuc[q]; c2 = gsequence[q]; c2_alt = gsequence_alt[q];
    if (c2 == '*') {
    } else if (c1_uc == c2 || c1_uc == c2_alt) {
      t->score += MATCH; t->nmatches += 1;
      sink_push(s, roffset + q, goffset + q, c1, DYNPROG_MATCH_COMP, c2, c2_alt, dpi);
    } else if (consistent[genestrand][(unsigned char) c1_uc][(unsigned char) c2] ||
               consistent[genestrand][(unsigned char) c1_uc][(unsigned char) c2_alt]) {
      t->score += MATCH; t->nmatches += 1;
      sink_push(s, roffset + q, goffset + q, c1, AMBIGUOUS_COMP, c2, c2_alt, dpi);
    } else {
      t->score += MISMATCH; t->nmismatches += 1;
      sink_push(s, roffset + q, goffset + q, c1, MISMATCH_COMP, c2, c2_alt, dpi);
    }
  }
  return t->nmismatches > 1 ? 0 : 1;
}

/* ---------------------------------------------------------------------------
 * SIMD-build fills (the "S" semantics of SURVEY §8: gmap.sse42/.avx2/.avx512
 * link dynprog_simd.c instead of Dynprog_standard).  Restated for the AVX2
 * layout (dynprog.h:128: 32 8-bit / 16 16-bit rows per block; the AVX-512
 * build uses the same dynprog code) with INFINITE_INITIAL_GAP_PENALTY
 * (dynprog.h:14).
 *
 * Dynprog_simd_8 / Dynprog_simd_16 (dynprog_simd.c:2987 / :6562) fill the
 * matrix in blocks of B rows.  Block rlo covers columns
 * [max(0, rlo-lband), min(rhigh+uband, glength)] for all B rows, in band or
 * not, with saturating 8/16-bit arithmetic; a scalar loop then adds the
 * vertical gaps inside the band (:3391-3478).  The row above a block
 * (matrix[c-1][rlo-1]) is read for every column of the block, including
 * columns the block above never wrote, and the traceback can walk into cells
 * no block wrote.  Those reads see whatever the Dynprog_T arena held before
 * the call (Dynprog_new never clears it, dynprog.c:686-731): the reference's
 * S output is not a function of its inputs alone.  This restatement, like the
 * engine, defines it on an arena that reads zero (DIAG) wherever the call
 * did not write -- what a fresh process's first call sees, and what the tests
 * pin by zeroing the reference's arenas (refh_poison_arenas) before each call.
 * ------------------------------------------------------------------------- */
static inline int
sat_add (int a, int b, int lo, int hi) {
  int s = a + b;
  return s < lo ? lo : (s > hi ? hi : s);
}

/* nt_to_int_array (dynprog.c:1012-1019): A C G T (either case) -> 0..3, anything else -> 4 ('N') */
static inline int
nt_to_int (int c) {
  switch (c) {
  case 'A': case 'a': return 0;
  case 'C': case 'c': return 1;
  case 'G': case 'g': return 2;
  case 'T': case 't': return 3;
  default: return 4;
  }
}

/* Full-band S fill (Dynprog_simd_8 when bits == 8, else Dynprog_simd_16).  Writes the three
   direction planes of traceback_std's layout (IDX(c, r), r <= rlength), DIAG where no block wrote. */
static void
simd_fill_full (int bits, const char *rsequence, const char *gsequence, const char *gsequence_alt,
                int rlength, int glength, int mismatchtype, int open, int extend, int lband, int uband,
                int late, int revp, signed char *dirs) {
  const int B = (bits == 8) ? 32 : 16;
  const int NEG = (bits == 8) ? -128 : -32768, POS = (bits == 8) ? 127 : 32767;
  const int ceil = ((rlength + B) / B) * B;  /* rlength_ceil: the arena's column pitch */
  const size_t cells = (size_t) (glength + 1) * (size_t) ceil;
  size_t plane = (size_t) (glength + 1) * (size_t) (rlength + 1);
  short (*pd)[128] = pairdistance[mismatchtype];
  static const char acgtn[5] = {'A', 'C', 'G', 'T', 'N'};
  int *mat = (int *) calloc(cells, sizeof(int));            /* Score8/16 matrix, zeroed arena */
  signed char *dn = (signed char *) calloc(cells, 1), *de = (signed char *) calloc(cells, 1);
  signed char *df = (signed char *) calloc(cells, 1);        /* Fgap is calloc'ed by the call itself */
  int *ps = (int *) malloc((size_t) 5 * ceil * sizeof(int));  /* pairscores[5][rlength_ceil] */
  int *FF = (int *) malloc((size_t) (glength + 1) * sizeof(int));
  int H[32], E[32], Hs[32], Hn[32];
  int rlo, rhigh, c, i, k, r, na1, na2, na2a, X, T1, rlo_calc, rhigh_calc, c_gap, last_nogap, score;

  for (k = 0; k < 5; k++) {
    for (r = 0; r < ceil; r++) {
      if (r == 0) na1 = 'N';
      else if (r <= rlength) na1 = (unsigned char) (revp ? rsequence[1 - r] : rsequence[r - 1]);
      else { ps[k * ceil + r] = 0; continue; }  /* past rlength: never reaches rows <= rlength */
      ps[k * ceil + r] = pd[na1][(int) acgtn[k]];
    }
  }

  for (rlo = 0; rlo <= rlength; rlo += B) {
    rhigh = (rlo + B - 1 > rlength) ? rlength : rlo + B - 1;
    c = (rlo - lband < 0) ? 0 : rlo - lband;
    for (i = 0; i < B; i++) {
      E[i] = late ? NEG : NEG + 1;
      H[i] = NEG - open;                       /* "compensate for T1 = H + open" */
    }
    for (; c <= rhigh + uband && c <= glength; c++) {
      int *col = mat + (size_t) c * ceil;
      if (c == 0) X = (rlo == 0) ? 0 : NEG;
      else X = (rlo == 0) ? NEG : mat[(size_t) (c - 1) * ceil + rlo - 1];
      na2 = na2a = 4;
      if (c > 0) {
        na2 = nt_to_int((unsigned char) (revp ? gsequence[1 - c] : gsequence[c - 1]));
        na2a = nt_to_int((unsigned char) (revp ? gsequence_alt[1 - c] : gsequence_alt[c - 1]));
      }
      for (i = 0; i < B; i++) {
        int p, pa, Hd;
        /* EGAP */
        T1 = sat_add(H[i], open, NEG, POS);
        de[(size_t) c * ceil + rlo + i] = (late ? (E[i] >= T1) : (E[i] > T1)) ? HORIZ : DIAG;
        E[i] = sat_add(E[i] > T1 ? E[i] : T1, extend, NEG, POS);
        /* NOGAP: H shifted down one row, row rlo from the row above the block */
        Hs[i] = (i == 0) ? X : H[i - 1];
        if (c == 0) p = (rlo + i == 0) ? 0 : NEG;  /* pairscores_col0 */
        else {
          p = ps[na2 * ceil + rlo + i];
          pa = ps[na2a * ceil + rlo + i];
          if (pa > p) p = pa;
        }
        Hd = sat_add(Hs[i], p, NEG, POS);
        dn[(size_t) c * ceil + rlo + i] = (late ? (E[i] >= Hd) : (E[i] > Hd)) ? HORIZ : DIAG;
        Hn[i] = Hd > E[i] ? Hd : E[i];
        col[rlo + i] = Hn[i];
      }
      /* F loop (:3391-3478) */
      rlo_calc = (rlo < c - uband) ? c - uband : rlo;
      if ((rhigh_calc = rhigh) >= c + lband) {
        rhigh_calc = c + lband;
        if (c > 0) {  /* bottom row: diagonal only, so no path leaves the band below */
          int p = ps[na2 * ceil + rhigh_calc], pa = ps[na2a * ceil + rhigh_calc];
          if (pa > p) p = pa;
          score = mat[(size_t) (c - 1) * ceil + rhigh_calc - 1] + p;
          col[rhigh_calc] = score < NEG ? NEG : (score > POS ? POS : score);
          de[(size_t) c * ceil + rhigh_calc] = DIAG;
          dn[(size_t) c * ceil + rhigh_calc] = DIAG;
        }
      }
      if (rlo == 0 || c >= rlo + uband) {
        c_gap = NEG_INFINITY_32;
        last_nogap = NEG_INFINITY_32;
      } else {
        c_gap = FF[c];
        last_nogap = col[rlo_calc - 1];
      }
      if ((r = rlo_calc) == c - uband) {  /* top of the band: no vertical gap into it */
        c_gap = last_nogap + open + extend;
        last_nogap = col[r];
        r++;
      }
      for (; r <= rhigh_calc; r++) {
        score = last_nogap + open;
        if (late ? (c_gap >= score) : (c_gap > score)) {
          c_gap += extend;
          df[(size_t) c * ceil + r] = VERT;
        } else {
          c_gap = score + extend;
        }
        last_nogap = col[r];
        if (late ? (c_gap >= last_nogap) : (c_gap > last_nogap)) {
          last_nogap = c_gap;
          col[r] = c_gap < NEG ? NEG : c_gap;
          dn[(size_t) c * ceil + r] = VERT;
        }
      }
      FF[c] = c_gap;
      for (i = 0; i < B; i++) H[i] = col[rlo + i];  /* reload after the F loop */
    }
  }

  memset(dirs, DIAG, 3 * plane);
  for (c = 0; c <= glength; c++) {
    for (r = 0; r <= rlength; r++) {
      dirs[IDX(c, r)] = dn[(size_t) c * ceil + r];
      dirs[plane + IDX(c, r)] = de[(size_t) c * ceil + r];
      dirs[2 * plane + IDX(c, r)] = df[(size_t) c * ceil + r];
    }
  }
  free(mat); free(dn); free(de); free(df); free(ps); free(FF);
}

/* Triangle fills of the SIMD builds: Dynprog_simd_8_upper / _16_upper (dynprog_simd.c:4304 /
   7714) and Dynprog_simd_8_lower / _16_lower (:5340 / :8586), AVX2 layout (B = 32 / 16 lanes).
   upper: matrix[c][r] for c >= r, horizontal gaps only; block rlo (B rows) covers columns
   [rlo, min(rhigh + uband, glength)].  lower: matrix[r][c] for r >= c, vertical gaps only,
   vectors along the genome; block clo (B columns) covers rows [clo, min(chigh + lband, rlength)].
   In both, E_mask keeps the gap of lane i at NEG until the lane is strictly off the diagonal
   (_MM_ADD_EPI8(E_mask, E_infinity) wraps 1 + POS to NEG), and the diagonal cell's directions
   are forced DIAG after the store.  Pair scores: upper scores query row r against genome class
   k (pairdistance[query char][ACGTN[k]], row 0 'N'); lower scores query class k against the
   genome column, max over the alternate allele (pairdistance[ACGTN[k]][g]), column 0 against
   byte 4 in the 8-bit fill, 'N' in the 16-bit one; scores past rlength (upper) / glength (lower) are
   uninitialised in the reference and read 0 here (they only reach cells outside the matrix).
   Output in traceback_std's layout (IDX(c, r), r <= rlength, c <= glength): score matrix and the
   three planes (upper: nogap HORIZ / Egap HORIZ; lower: nogap VERT / Fgap VERT), 0 / DIAG where
   no block wrote (a zeroed arena, as simd_fill_full). */
static void
simd_fill_ud (int bits, int upperp, const char *rsequence, const char *gsequence, const char *gsequence_alt,
              int rlength, int glength, int mismatchtype, int open, int extend, int band, int late, int revp,
              int *matrix, signed char *dirs) {
  const int B = (bits == 8) ? 32 : 16;
  const int NEG = (bits == 8) ? -128 : -32768, POS = (bits == 8) ? 127 : 32767;
  const int nrow = upperp ? rlength : glength;   /* lanes index rows (upper) / columns (lower) */
  const int ncol = upperp ? glength : rlength;   /* steps walk columns (upper) / rows (lower) */
  const int ceil = ((nrow + B) / B) * B;
  const size_t plane = (size_t) (glength + 1) * (size_t) (rlength + 1);
  signed char *dnogap = dirs, *dE = dirs + plane, *dF = dirs + 2 * plane;
  short (*pd)[128] = pairdistance[mismatchtype];
  static const char acgtn[5] = {'A', 'C', 'G', 'T', 'N'};
  int *mat = (int *) calloc((size_t) (ncol + 1) * ceil, sizeof(int));      /* [step][lane-row] */
  signed char *dn = (signed char *) calloc((size_t) (ncol + 1) * ceil, 1);
  signed char *de = (signed char *) calloc((size_t) (ncol + 1) * ceil, 1);
  int *ps = (int *) calloc((size_t) 5 * ceil, sizeof(int));                /* pairscores[5][ceil] */
  int H[32], E[32], Hs[32], mask[32];
  int lo, hi, x, i, k, na, p, T1, Hd, X;
  size_t at;

  for (k = 0; k < 5; k++) {
    for (i = 0; i <= nrow && i < ceil; i++) {
      int s1, s2;
      if (upperp) {
        int na1 = (i == 0) ? 'N' : (unsigned char) (revp ? rsequence[1 - i] : rsequence[i - 1]);
        ps[k * ceil + i] = pd[na1][(int) acgtn[k]];
      } else if (i == 0) {
        /* column 0: the 8-bit fill indexes byte 4 (dynprog_simd.c:5459), the 16-bit one 'N' (:8690) */
        ps[k * ceil + i] = pd[(int) acgtn[k]][bits == 8 ? 4 : 'N'];
      } else {
        int g = (unsigned char) (revp ? gsequence[1 - i] : gsequence[i - 1]);
        int ga = (unsigned char) (revp ? gsequence_alt[1 - i] : gsequence_alt[i - 1]);
        s1 = pd[(int) acgtn[k]][g];
        s2 = pd[(int) acgtn[k]][ga];
        ps[k * ceil + i] = s1 > s2 ? s1 : s2;
      }
    }
  }

  for (lo = 0; lo <= nrow; lo += B) {
    hi = (lo + B - 1 > nrow) ? nrow : lo + B - 1;
    for (i = 0; i < B; i++) {
      E[i] = late ? NEG : NEG + 1;
      H[i] = NEG - open;               /* "compensate for T1 = H + open" */
      mask[i] = 1;
    }
    for (x = lo; x <= hi + band && x <= ncol; x++) {
      if (x == 0) {
        na = 4;
      } else if (upperp) {
        na = nt_to_int((unsigned char) (revp ? gsequence[1 - x] : gsequence[x - 1]));
      } else {
        na = nt_to_int((unsigned char) (revp ? rsequence[1 - x] : rsequence[x - 1]));
      }
      if (x == 0) X = 0;
      else if (lo == 0) X = NEG;
      else X = mat[(size_t) (x - 1) * ceil + lo - 1];
      for (i = 0; i < B; i++) {
        at = (size_t) x * ceil + lo + i;
        if (mask[i]) E[i] = NEG;                          /* min(E, wrap(1 + POS)) */
        T1 = sat_add(H[i], open, NEG, POS);
        de[at] = (late ? (E[i] >= T1) : (E[i] > T1)) ? -1 : 0;
        E[i] = sat_add(E[i] > T1 ? E[i] : T1, extend, NEG, POS);
        if (mask[i]) E[i] = NEG;
        Hs[i] = (i == 0) ? X : H[i - 1];
      }
      for (i = 0; i < B; i++) {
        at = (size_t) x * ceil + lo + i;
        if (upperp) {
          p = ps[na * ceil + lo + i];
          {
            int na_alt = (x == 0) ? 4 : nt_to_int((unsigned char) (revp ? gsequence_alt[1 - x] : gsequence_alt[x - 1]));
            int pa = ps[na_alt * ceil + lo + i];
            if (pa > p) p = pa;
          }
        } else {
          p = ps[na * ceil + lo + i];
        }
        Hd = sat_add(Hs[i], p, NEG, POS);
        dn[at] = (late ? (E[i] >= Hd) : (E[i] > Hd)) ? -1 : 0;
        H[i] = Hd > E[i] ? Hd : E[i];
        mat[at] = H[i];
      }
      if (hi >= x) {                                       /* diagonal forced DIAG */
        de[(size_t) x * ceil + x] = 0;
        dn[(size_t) x * ceil + x] = 0;
      }
      for (i = B - 1; i > 0; i--) mask[i] = mask[i - 1];
      mask[0] = 0;
    }
  }

  memset(matrix, 0, plane * sizeof(int));
  memset(dirs, DIAG, 3 * plane);
  for (x = 0; x <= ncol; x++) {
    for (i = 0; i <= nrow; i++) {
      at = (size_t) x * ceil + i;
      if (upperp) {          /* x = c, i = r */
        matrix[IDX(x, i)] = mat[at];
        dnogap[IDX(x, i)] = dn[at] ? HORIZ : DIAG;
        dE[IDX(x, i)] = de[at] ? HORIZ : DIAG;
      } else {               /* x = r, i = c */
        matrix[IDX(i, x)] = mat[at];
        dnogap[IDX(i, x)] = dn[at] ? VERT : DIAG;
        dF[IDX(i, x)] = de[at] ? VERT : DIAG;
      }
    }
  }
  free(mat); free(dn); free(de); free(ps);
}

static void
reverse_pairs (OrcPair *p, int n) {
  int i, j;
  OrcPair t;
  for (i = 0, j = n - 1; i < j; i++, j--) { t = p[i]; p[i] = p[j]; p[j] = t; }
}

int
orc_single_gap (const char *rsequence, const char *rsequenceuc, int rlength, int glength,
                int roffset, int goffset, unsigned int chroffset, unsigned int chrhigh,
                int watsonp, int genestrand, int jump_late_p, int extraband_single, int widebandp,
                double defect_rate, int dynprogindex, int *scalars, OrcPair *out, int max_pairs) {
  int mismatchtype, open, extend, lband, uband, n;
  char *gseq, *gseq_alt;
  int *matrix;
  signed char *dirs;
  PairSink sink = {out, 0, max_pairs};
  Tally t = {0, 0, 0, 0, 0};
  int dpi_next = dynprogindex + (dynprogindex > 0 ? +1 : -1);

  if (defect_rate < DEFECT_HIGHQ) mismatchtype = HIGHQ;
  else if (defect_rate < DEFECT_MEDQ) mismatchtype = MEDQ;
  else mismatchtype = LOWQ;

  if (g_user_dynprog_p) { open = g_user_open; extend = g_user_extend; }
  else if (defect_rate < DEFECT_HIGHQ) { open = SINGLE_OPEN_HIGHQ; extend = SINGLE_EXTEND_HIGHQ; }
  else if (defect_rate < DEFECT_MEDQ) { open = SINGLE_OPEN_MEDQ; extend = SINGLE_EXTEND_MEDQ; }
  else { open = SINGLE_OPEN_LOWQ; extend = SINGLE_EXTEND_LOWQ; }

  if (rlength <= 0 || glength <= 0 || rlength > ORC_MAX_RLENGTH || glength > ORC_MAX_GLENGTH) {
    scalars[0] = dpi_next; scalars[1] = NEG_INFINITY_32;
    scalars[2] = scalars[3] = scalars[4] = scalars[5] = 0;
    return -1;
  }

  gseq = (char *) malloc(glength + 1);
  gseq_alt = (char *) malloc(glength + 1);
  if (watsonp) orc_get_segment(1, chroffset + (unsigned int) goffset, glength, chrhigh, 0, gseq, gseq_alt);
  else orc_get_segment(0, chrhigh - (unsigned int) goffset + 1, glength, chroffset, 1, gseq, gseq_alt);

  if (gseq[0] == '\0') {
    scalars[0] = dynprogindex; scalars[1] = NEG_INFINITY_32;
    scalars[2] = scalars[3] = scalars[4] = scalars[5] = 0;
    free(gseq); free(gseq_alt);
    return -1;
  }
  if (glength == rlength) {
    if (single_gap_simple(&sink, &t, rsequence, rsequenceuc, rlength, gseq, gseq_alt, roffset, goffset,
                          genestrand, dynprogindex)) {
      /* list order = reverse of push order; no List_reverse on this path */
      n = sink.n < max_pairs ? sink.n : max_pairs;
      reverse_pairs(out, n);
      scalars[0] = dpi_next; scalars[1] = t.score; scalars[2] = t.nmatches; scalars[3] = t.nmismatches;
      scalars[4] = 0; scalars[5] = 0;
      free(gseq); free(gseq_alt);
      return sink.n > 0 ? sink.n : -1; /* an empty List_T is NULL */
    }
    sink.n = 0;
    t.score = t.nmatches = t.nmismatches = 0;
  }

  compute_bands(&lband, &uband, rlength, glength, extraband_single, widebandp);
  matrix = (int *) malloc((size_t) (glength + 1) * (rlength + 1) * sizeof(int));
  dirs = (signed char *) malloc((size_t) 3 * (glength + 1) * (rlength + 1));
  if (g_simd) {
    /* dynprog_single.c:593-631: 8-bit fill when both lengths are below use8p_size */
    int bits = (rlength < use8p_size[mismatchtype] && glength < use8p_size[mismatchtype]) ? 8 : 16;
    simd_fill_full(bits, rsequence, gseq, gseq_alt, rlength, glength, mismatchtype, open, extend, lband, uband,
                   jump_late_p, /*revp*/0, dirs);
  } else {
    orc_standard_fill(rsequence, gseq, gseq_alt, rlength, glength, mismatchtype, open, extend, lband, uband,
                      jump_late_p, /*revp*/0, /*saturation*/NEG_INFINITY_32, 1, 1, matrix, dirs);
  }
  traceback_std(&sink, &t, dirs, rlength, glength, rlength, glength, rsequence, rsequenceuc, gseq, gseq_alt,
                roffset, goffset, /*revp*/0, chroffset, chrhigh, watsonp, genestrand, dynprogindex);
  /* pushes prepend; List_reverse (dynprog_single.c:675) => list order == push order */
  scalars[0] = dpi_next;
  scalars[1] = t.score;
  scalars[2] = t.nmatches; scalars[3] = t.nmismatches; scalars[4] = t.nopens; scalars[5] = t.nindels;
  free(matrix); free(dirs); free(gseq); free(gseq_alt);
  return sink.n > 0 ? sink.n : -1; /* an empty List_T is NULL */
}

/* ---------------------------------------------------------------------------
 * Dynprog_end5_gap / Dynprog_end3_gap (dynprog_end.c:1294-1647 / 1924-2247),
 * nosimd build: ENDQ scores, END_OPEN/EXTEND penalties (dynprog_end.c:68-74),
 * find_best_endpoint_std / _to_queryend_indels_std / _nogaps
 * (dynprog_end.c:297-587), traceback_nogaps (:649), then removal of INDEL
 * pairs at the far end.  qbuf/qucbuf + qpos is the reference's
 * (rev_)rsequence pointer: for end5 it points at the LAST query character
 * and the fill walks backwards (revp).
 * ------------------------------------------------------------------------- */
#define END_OPEN_HIGHQ -10
#define END_OPEN_MEDQ -8
#define END_OPEN_LOWQ -6
#define END_EXTEND -2
enum { QUERYEND_GAP = 0, QUERYEND_INDELS = 1, QUERYEND_NOGAPS = 2, BEST_LOCAL = 3 };

static void
find_best_endpoint_std (int *finalscore, int *bestr, int *bestc, const int *matrix, int rlength, int glength,
                        int lband, int uband, int late) {
  int bestscore = 0, r, c, clo, chigh;
  *bestr = *bestc = 0;
  for (r = 1; r <= rlength; r++) {
    if ((clo = r - lband) < 1) clo = 1;
    if ((chigh = r + uband) > glength) chigh = glength;
    for (c = clo; c <= chigh; c++) {
      if (prefer(matrix[IDX(c, r)], bestscore, late)) { *bestr = r; *bestc = c; bestscore = matrix[IDX(c, r)]; }
    }
  }
  *finalscore = bestscore;
}

static void
find_best_endpoint_to_queryend_indels_std (int *finalscore, int *bestr, int *bestc, const int *matrix, int rlength,
                                           int glength, int lband, int uband, int late) {
  int bestscore = NEG_INFINITY_32, r, c, clo, chigh;
  *bestr = r = rlength;
  *bestc = 0;
  if ((clo = r - lband) < 1) clo = 1;
  if ((chigh = r + uband) > glength) chigh = glength;
  for (c = clo; c <= chigh; c++) {
    if (prefer(matrix[IDX(c, r)], bestscore, late)) { *bestr = r; *bestc = c; bestscore = matrix[IDX(c, r)]; }
  }
  *finalscore = bestscore;
}

/* find_best_endpoint_8/_16 (dynprog_end.c:144/220) and
   find_best_endpoint_to_queryend_indels_8/_16 (:359/437): the same scans over the two
   triangles, lower[r][c] for c < r (this loop is bounded by r, not by chigh), then upper[c][r]
   for r <= c <= chigh; bestscore starts at 0 (resp. NEG_INFINITY_8/16) in the fill's width. */
static void
find_best_endpoint_ud (int *finalscore, int *bestr, int *bestc, const int *mupper, const int *mlower,
                       int rlength, int glength, int lband, int uband, int late, int indels, int neg) {
  int bestscore = indels ? neg : 0, r, c, clo, chigh, r0;
  *bestr = *bestc = 0;
  r0 = 1;
  if (indels) { *bestr = r0 = rlength; }
  for (r = r0; r <= rlength; r++) {
    if ((clo = r - lband) < 1) clo = 1;
    if ((chigh = r + uband) > glength) chigh = glength;
    for (c = clo; c < r; c++) {
      if (prefer(mlower[IDX(c, r)], bestscore, late)) { *bestr = r; *bestc = c; bestscore = mlower[IDX(c, r)]; }
    }
    for (; c <= chigh; c++) {
      if (prefer(mupper[IDX(c, r)], bestscore, late)) { *bestr = r; *bestc = c; bestscore = mupper[IDX(c, r)]; }
    }
  }
  *finalscore = bestscore;
}

/* traceback_nogaps (dynprog_end.c:649) */
static void
traceback_nogaps (PairSink *s, Tally *t, int r, int c, const char *rsequence, const char *rsequenceuc,
                  const char *gsequence, const char *gsequence_alt, int queryoffset, int genomeoffset,
                  int genestrand, int revp, int dpi) {
  int querycoord, genomecoord;
  char c1, c1_uc, c2, c2_alt;
  while (r > 0 && c > 0) {
    querycoord = r - 1;
    genomecoord = c - 1;
    if (revp) { querycoord = -querycoord; genomecoord = -genomecoord; }
    c1 = rsequence[querycoord]; c1_uc = rsequenceuc[querycoord];
    c2 = gsequence[genomecoord]; c2_alt = gsequence_alt[genomecoord];
    if (c2 == '*') {
    } else if (c1_uc == c2 || c1_uc == c2_alt) {
      t->score += MATCH; t->nmatches += 1;
      sink_push(s, queryoffset + querycoord, genomeoffset + genomecoord, c1, DYNPROG_MATCH_COMP, c2, c2_alt, dpi);
    } else if (consistent[genestrand][(unsigned char) c1_uc][(unsigned char) c2] ||
               consistent[genestrand][(unsigned char) c1_uc][(unsigned char) c2_alt]) {
      t->score += MATCH; t->nmatches += 1;
      sink_push(s, queryoffset + querycoord, genomeoffset + genomecoord, c1, AMBIGUOUS_COMP, c2, c2_alt, dpi);
    } else {
      t->score += MISMATCH; t->nmismatches += 1;
      sink_push(s, queryoffset + querycoord, genomeoffset + genomecoord, c1, MISMATCH_COMP, c2, c2_alt, dpi);
    }
    r--; c--;
  }
}

int
orc_end_gap (int end3p, const char *qbuf, const char *qucbuf, int qpos, int rlength, int glength,
             int roffset, int goffset, unsigned int chroffset, unsigned int chrhigh,
             int watsonp, int genestrand, int jump_late_p, int extraband_end, double defect_rate,
             int endalign, int require_pos_score_p, int dynprogindex, int *scalars, OrcPair *out, int max_pairs) {
  const char *rsequence = qbuf + qpos, *rsequenceuc = qucbuf + qpos;
  int open, extend, lband = 0, uband = 0, bestr = 0, bestc = 0, finalscore = 0, n, i, first, revp = !end3p;
  int late = end3p ? jump_late_p : !jump_late_p;
  char *gseq, *gseq_alt;
  const char *gptr, *gptr_alt;
  int *matrix = NULL;
  signed char *dirs = NULL;
  PairSink sink = {out, 0, max_pairs};
  Tally t = {0, 0, 0, 0, 0};

  if (g_user_dynprog_p) { open = g_user_open; extend = g_user_extend; }
  else if (defect_rate < DEFECT_HIGHQ) { open = END_OPEN_HIGHQ; extend = END_EXTEND; }
  else if (defect_rate < DEFECT_MEDQ) { open = END_OPEN_MEDQ; extend = END_EXTEND; }
  else { open = END_OPEN_LOWQ; extend = END_EXTEND; }

  scalars[0] = dynprogindex;
  scalars[1] = scalars[2] = scalars[3] = scalars[4] = scalars[5] = 0;
  if (rlength <= 0) return -1;
  if (endalign != QUERYEND_NOGAPS && rlength > ORC_MAX_RLENGTH) rlength = ORC_MAX_RLENGTH;
  if (!end3p && goffset < 0) return -1;
  if (glength <= 0) return -1;
  if (endalign != QUERYEND_NOGAPS && glength > ORC_MAX_GLENGTH) glength = ORC_MAX_GLENGTH;

  gseq = (char *) malloc(glength + 1);
  gseq_alt = (char *) malloc(glength + 1);
  if (end3p) {
    if (watsonp) orc_get_segment(1, chroffset + (unsigned int) goffset, glength, chrhigh, 0, gseq, gseq_alt);
    else orc_get_segment(0, chrhigh - (unsigned int) goffset + 1, glength, chroffset, 1, gseq, gseq_alt);
    gptr = gseq; gptr_alt = gseq_alt;
  } else {
    if (watsonp) orc_get_segment(0, chroffset + (unsigned int) goffset + 1, glength, chroffset, 0, gseq, gseq_alt);
    else orc_get_segment(1, chrhigh - (unsigned int) goffset, glength, chrhigh, 1, gseq, gseq_alt);
    gptr = &gseq[glength - 1]; gptr_alt = &gseq_alt[glength - 1];
  }
  if (gseq[0] == '\0') { free(gseq); free(gseq_alt); return -1; }

  if (g_simd && (endalign == QUERYEND_GAP || endalign == BEST_LOCAL || endalign == QUERYEND_INDELS)) {
    /* dynprog_end.c:1406-1510 / 2027-2140: 8-bit triangles when either length is below use8p_size */
    int bits = (rlength < use8p_size[ENDQ] || glength < use8p_size[ENDQ]) ? 8 : 16;
    size_t plane;
    compute_bands(&lband, &uband, rlength, glength, extraband_end, endalign != QUERYEND_INDELS);
    plane = (size_t) (glength + 1) * (rlength + 1);
    matrix = (int *) malloc(2 * plane * sizeof(int));
    dirs = (signed char *) malloc((size_t) 6 * plane);
    if (rlength > glength + 1) {
      /* outside the domain: the lower-triangle scans would read columns past glength, which the
         reference fills from uninitialised pair scores (stage3.c always passes glength >= rlength) */
      free(matrix); free(dirs); free(gseq); free(gseq_alt);
      return -3;
    }
    simd_fill_ud(bits, 1, end3p ? rsequenceuc : rsequence, gptr, gptr_alt, rlength, glength, ENDQ, open, extend,
                 uband, late, revp, matrix, dirs);
    simd_fill_ud(bits, 0, end3p ? rsequenceuc : rsequence, gptr, gptr_alt, rlength, glength, ENDQ, open, extend,
                 lband, late, revp, matrix + plane, dirs + 3 * plane);
    find_best_endpoint_ud(&finalscore, &bestr, &bestc, matrix, matrix + plane, rlength, glength, lband, uband,
                          late, endalign == QUERYEND_INDELS, bits == 8 ? -128 : -32768);
  } else if (endalign == QUERYEND_GAP || endalign == BEST_LOCAL || endalign == QUERYEND_INDELS) {
    compute_bands(&lband, &uband, rlength, glength, extraband_end, endalign != QUERYEND_INDELS);
    matrix = (int *) malloc((size_t) (glength + 1) * (rlength + 1) * sizeof(int));
    dirs = (signed char *) malloc((size_t) 3 * (glength + 1) * (rlength + 1));
    /* end3 scores the upper-cased query, end5 the query as given */
    orc_standard_fill(end3p ? rsequenceuc : rsequence, gptr, gptr_alt, rlength, glength, ENDQ, open, extend,
                      lband, uband, late, revp, NEG_INFINITY_32, 1, 1, matrix, dirs);
    if (endalign == QUERYEND_INDELS)
      find_best_endpoint_to_queryend_indels_std(&finalscore, &bestr, &bestc, matrix, rlength, glength, lband, uband, late);
    else
      find_best_endpoint_std(&finalscore, &bestr, &bestc, matrix, rlength, glength, lband, uband, late);
  } else if (endalign == QUERYEND_NOGAPS) {
    bestr = bestc = glength < rlength ? glength : rlength;
  } else {
    free(gseq); free(gseq_alt);
    return -2;
  }

  if (endalign == QUERYEND_NOGAPS) {
    traceback_nogaps(&sink, &t, bestr, bestc, rsequence, rsequenceuc, gptr, gptr_alt, roffset, goffset,
                     genestrand, revp, dynprogindex);
  } else if (require_pos_score_p) {
    /* *traceback_score was just zeroed, so this always skips (dynprog_end.c:1572) */
  } else if (g_simd) {
    /* Dynprog_traceback_{8,16}_upper when bestc >= bestr, else _lower (dynprog_end.c:1574-1610) */
    size_t plane = (size_t) (glength + 1) * (rlength + 1);
    int up = bestc >= bestr;
    traceback_mode(&sink, &t, up ? dirs : dirs + 3 * plane, rlength, glength, bestr, bestc, rsequence, rsequenceuc,
                   gptr, gptr_alt, roffset, goffset, revp, chroffset, chrhigh, watsonp, genestrand, dynprogindex,
                   up ? 1 : 2);
  } else {
    traceback_std(&sink, &t, dirs, rlength, glength, bestr, bestc, rsequence, rsequenceuc, gptr, gptr_alt,
                  roffset, goffset, revp, chroffset, chrhigh, watsonp, genestrand, dynprogindex);
  }
  scalars[0] = dynprogindex + (dynprogindex > 0 ? +1 : -1);
  scalars[1] = t.score; scalars[2] = t.nmatches; scalars[3] = t.nmismatches;
  scalars[4] = t.nopens; scalars[5] = t.nindels;
  free(matrix); free(dirs); free(gseq); free(gseq_alt);

  if ((endalign == QUERYEND_GAP || endalign == BEST_LOCAL) && (t.nmatches + 1) < t.nmismatches) {
    scalars[1] = 0;
    return -1;
  }
  /* push order == List_reverse(pairs); drop INDEL pairs at its head (the far end) */
  n = sink.n < max_pairs ? sink.n : max_pairs;
  for (first = 0; first < n && out[first].comp == INDEL_COMP; first++) ;
  for (i = first; i < n; i++) out[i - first] = out[i];
  n -= first;
  if (!end3p) reverse_pairs(out, n); /* end5 returns List_reverse once more */
  return n > 0 ? n : -1;
}

/* ---------------------------------------------------------------------------
 * Dynprog_end5_splicejunction / Dynprog_end3_splicejunction (dynprog_end.c:1653 /
 * 2249), nosimd build: the end-gap fill (Dynprog_standard, ENDQ, END penalties,
 * wide band) against the caller's junction string instead of the genome,
 * find_best_endpoint_to_queryend_indels_std, and -- when the best score is not
 * negative -- traceback_local_std (:1138) twice: the far piece (columns past
 * contlength, genome positions from goffset_far), the known-splice gap holder,
 * then the anchor piece (goffset_anchor).  Genome skips take their characters
 * from the junction string (Pairpool_add_genomeskip with a genomesequence,
 * pairpool.c:1145).  scalars[0..7] = dynprogindex(after), traceback_score,
 * missscore, nmatches, nmismatches, nopens, nindels, index of the known gap
 * holder in the returned list (-1: none); out-parameters the reference leaves
 * unwritten stay ORC_UNSET.
 * ------------------------------------------------------------------------- */
#define ORC_UNSET_SJ (-2147483647 - 1)

/* Pairpool_add_genomeskip with the junction string as genomesequence */
static int
add_genomeskip_seq (PairSink *s, int r, int c, int dist, const char *gsequence, int queryoffset, int genomeoffset,
                    int revp, int dpi) {
  int j, querycoord = r - 1, left = c - dist, right = c - 1, t, genomecoord, step;
  if (revp) { querycoord = -querycoord; t = left; left = -right; right = -t; step = +1; } else { step = -1; }
  if (dist >= MICROINTRON_LENGTH) {
    sink_gapholder(s, 0, dist);
    return 0;
  }
  genomecoord = revp ? left : right;
  for (j = 0; j < dist; j++) {
    sink_push(s, queryoffset + querycoord, genomeoffset + genomecoord, ' ', INDEL_COMP, gsequence[genomecoord],
              gsequence[genomecoord], dpi);
    genomecoord += step;
  }
  return 1;
}

/* One gap step of traceback_local_std at cell (r, c): nothing on DIAG, else the E or F chain
   (the reference's `c > 1` / `r > 1` guards) and its records. */
static void
local_gap (PairSink *s, Tally *t, const signed char *dirs, int rlength, int glength, int *rp, int *cp,
           const char *rsequence, const char *gsequence, int queryoffset, int genomeoffset, int revp, int dpi) {
  size_t plane = (size_t) (glength + 1) * (size_t) (rlength + 1);
  const signed char *dnogap = dirs, *dE = dirs + plane, *dF = dirs + 2 * plane;
  int r = *rp, c = *cp, dist = 1;
  signed char dir = dnogap[IDX(c, r)];
  if (dir == DIAG) return;
  if (dir == HORIZ) {
    while (c > 1 && dE[IDX(c, r)] != DIAG) { dist++; c--; }
    c--;
    if (add_genomeskip_seq(s, r, c + dist, dist, gsequence, queryoffset, genomeoffset, revp, dpi)) {
      t->score += TOPEN + dist * TINDEL;
      t->nopens += 1;
      t->nindels += dist;
    }
  } else {
    while (r > 1 && dF[IDX(c, r)] != DIAG) { dist++; r--; }
    r--;
    add_queryskip(s, r + dist, c, dist, rsequence, queryoffset, genomeoffset, revp, dpi);
    t->score += QOPEN + dist * QINDEL;
    t->nopens += 1;
    t->nindels += dist;
  }
  *rp = r;
  *cp = c;
}

/* traceback_local_std (dynprog_end.c:1138): stops once the column reaches endc (or the row 0) */
static void
traceback_local (PairSink *s, Tally *t, const signed char *dirs, int rlength, int glength, int *rp, int *cp, int endc,
                 const char *rsequence, const char *rsequenceuc, const char *gsequence, int queryoffset,
                 int genomeoffset, int revp, int genestrand, int dpi) {
  int querycoord, genomecoord;
  char c1, c1_uc, c2;
  if (*cp > endc)
    local_gap(s, t, dirs, rlength, glength, rp, cp, rsequence, gsequence, queryoffset, genomeoffset, revp, dpi);
  while (*rp > 0 && *cp > endc) {
    querycoord = *rp - 1;
    genomecoord = *cp - 1;
    if (revp) { querycoord = -querycoord; genomecoord = -genomecoord; }
    c1 = rsequence[querycoord];
    c1_uc = rsequenceuc[querycoord];
    c2 = gsequence[genomecoord];
    if (c1_uc == c2) {
      t->score += MATCH; t->nmatches += 1;
      sink_push(s, queryoffset + querycoord, genomeoffset + genomecoord, c1, DYNPROG_MATCH_COMP, c2, c2, dpi);
    } else if (consistent[genestrand][(unsigned char) c1_uc][(unsigned char) c2]) {
      t->score += MATCH; t->nmatches += 1;
      sink_push(s, queryoffset + querycoord, genomeoffset + genomecoord, c1, AMBIGUOUS_COMP, c2, c2, dpi);
    } else {
      t->score += MISMATCH; t->nmismatches += 1;
      sink_push(s, queryoffset + querycoord, genomeoffset + genomecoord, c1, MISMATCH_COMP, c2, c2, dpi);
    }
    (*rp)--;
    (*cp)--;
    if (!(*rp == 0 && *cp == 0))
      local_gap(s, t, dirs, rlength, glength, rp, cp, rsequence, gsequence, queryoffset, genomeoffset, revp, dpi);
  }
}

int
orc_end_splicejunction (int end3p, const char *qbuf, const char *qucbuf, int qpos, const char *jbuf, int jpos,
                        int rlength, int glength, int roffset, int goffset_anchor, int goffset_far, int genestrand,
                        int jump_late_p, int extraband_end, double defect_rate, int contlength, int dynprogindex,
                        int *scalars, OrcPair *out, int max_pairs) {
  const char *rsequence = qbuf + qpos, *rsequenceuc = qucbuf + qpos, *gseq = jbuf + jpos;
  int open, extend, lband, uband, bestr, bestc, finalscore, n, i, first, known, revp = !end3p;
  int late = end3p ? jump_late_p : !jump_late_p;
  int *matrix;
  signed char *dirs;
  PairSink sink = {out, 0, max_pairs};
  Tally t = {0, 0, 0, 0, 0};

  if (g_user_dynprog_p) { open = g_user_open; extend = g_user_extend; }
  else if (defect_rate < DEFECT_HIGHQ) { open = END_OPEN_HIGHQ; extend = END_EXTEND; }
  else if (defect_rate < DEFECT_MEDQ) { open = END_OPEN_MEDQ; extend = END_EXTEND; }
  else { open = END_OPEN_LOWQ; extend = END_EXTEND; }

  scalars[0] = dynprogindex;
  for (i = 1; i < 7; i++) scalars[i] = ORC_UNSET_SJ;
  scalars[7] = -1;
  if (rlength <= 0 || rlength > ORC_MAX_RLENGTH || glength <= 0 || glength > ORC_MAX_GLENGTH) {
    scalars[1] = scalars[3] = scalars[4] = scalars[5] = scalars[6] = 0;
    scalars[2] = -100;
    return -1;
  }
  compute_bands(&lband, &uband, rlength, glength, extraband_end, 1);
  matrix = (int *) malloc((size_t) (glength + 1) * (rlength + 1) * sizeof(int));
  dirs = (signed char *) malloc((size_t) 3 * (glength + 1) * (rlength + 1));
  /* end3 scores the upper-cased query, end5 the query as given (as the end gaps) */
  orc_standard_fill(end3p ? rsequenceuc : rsequence, gseq, gseq, rlength, glength, ENDQ, open, extend, lband, uband,
                    late, revp, NEG_INFINITY_32, 1, 1, matrix, dirs);
  find_best_endpoint_to_queryend_indels_std(&finalscore, &bestr, &bestc, matrix, rlength, glength, lband, uband, late);
  if (finalscore < 0) {
    free(matrix); free(dirs);
    return -1;  /* "Need a reasonable alignment to call a splice": nothing written */
  }
  traceback_local(&sink, &t, dirs, rlength, glength, &bestr, &bestc, contlength, rsequence, rsequenceuc, gseq,
                  roffset, goffset_far, revp, genestrand, dynprogindex);
  known = sink.n;
  sink_gapholder(&sink, 0, end3p ? goffset_far - goffset_anchor : goffset_anchor - goffset_far);
  traceback_local(&sink, &t, dirs, rlength, glength, &bestr, &bestc, 0, rsequence, rsequenceuc, gseq,
                  roffset, goffset_anchor, revp, genestrand, dynprogindex);
  free(matrix); free(dirs);

  scalars[0] = dynprogindex + (dynprogindex > 0 ? +1 : -1);
  scalars[1] = t.score; scalars[2] = t.score - rlength * FULLMATCH;
  scalars[3] = t.nmatches; scalars[4] = t.nmismatches; scalars[5] = t.nopens; scalars[6] = t.nindels;
  /* push order == List_reverse(pairs); INDEL pairs at its head (the far end) dropped */
  n = sink.n < max_pairs ? sink.n : max_pairs;
  for (first = 0; first < n && out[first].comp == INDEL_COMP; first++) ;
  for (i = first; i < n; i++) out[i - first] = out[i];
  n -= first;
  known -= first;
  if (!end3p) {
    reverse_pairs(out, n); /* end5 returns List_reverse once more */
    known = n - 1 - known;
  }
  scalars[7] = known;
  return n;
}

/* ---------------------------------------------------------------------------
 * Dynprog_genome_gap (dynprog_genome.c:3288-3901), nosimd build, no splicing
 * IIT (Dynprog_genome_setup with splicing_iit NULL: get_known_splicesites
 * :405 adds nothing, so left_known/right_known stay 0 and
 * bridge_intron_gap_site_level :2469 is the bridge).  The MaxEnt splice-site
 * probabilities (Maxent_hr_*_prob, maxent_hr.c:27357-27600) are host inputs:
 * left_probs[c], c in [0, glengthL), and right_probs[c], c in [0, glengthR),
 * at the positions orc_genome_splice_sites gives (:2573-2660, :332-401).
 * ------------------------------------------------------------------------- */
#define PAIRED_OPEN_HIGHQ -8
#define PAIRED_OPEN_MEDQ -7
#define PAIRED_OPEN_LOWQ -6
#define PAIRED_EXTEND_HIGHQ -3
#define PAIRED_EXTEND_MEDQ -2
#define PAIRED_EXTEND_LOWQ -1
#define PROB_CEILING 0.85                /* dynprog_genome.c:82 */
#define GCAG_INTRON 8                    /* :98-103 */
#define ATAC_INTRON 4
#define FINAL_GCAG_INTRON 10
#define FINAL_ATAC_INTRON 8
#define CANONICAL_INTRON_HIGHQ 14        /* :109 */
#define FINAL_CANONICAL_INTRON_HIGHQ 16  /* :114 */
/* intron.h:11-35 */
#define LEFT_GT 0x21
#define LEFT_GC 0x10
#define LEFT_AT 0x08
#define LEFT_CT 0x06
#define RIGHT_AG 0x30
#define RIGHT_AC 0x0C
#define RIGHT_GC 0x02
#define RIGHT_AT 0x01
#define GTAG_FWD 0x20
#define GCAG_FWD 0x10
#define ATAC_FWD 0x08
#define GTAG_REV 0x04
#define GCAG_REV 0x02
#define ATAC_REV 0x01
#define ORC_UNSET (-2147483647 - 1)

/* intron_score_setup (dynprog_genome.c:144): [direction class][finalp][leftdi & rightdi];
   class 0 = sense (cdna_direction > 0), 1 = antisense (< 0), 2 = either. */
static int intron_score[3][2][64];

static void
intron_score_setup (void) {
  memset(intron_score, 0, sizeof(intron_score));
  intron_score[0][1][GTAG_FWD] = FINAL_CANONICAL_INTRON_HIGHQ;
  intron_score[0][1][GCAG_FWD] = FINAL_GCAG_INTRON;
  intron_score[0][1][ATAC_FWD] = FINAL_ATAC_INTRON;
  intron_score[0][0][GTAG_FWD] = CANONICAL_INTRON_HIGHQ;
  intron_score[0][0][GCAG_FWD] = GCAG_INTRON;
  intron_score[0][0][ATAC_FWD] = ATAC_INTRON;
  intron_score[1][1][GTAG_REV] = FINAL_CANONICAL_INTRON_HIGHQ;
  intron_score[1][1][GCAG_REV] = FINAL_GCAG_INTRON;
  intron_score[1][1][ATAC_REV] = FINAL_ATAC_INTRON;
  intron_score[1][0][GTAG_REV] = CANONICAL_INTRON_HIGHQ;
  intron_score[1][0][GCAG_REV] = GCAG_INTRON;
  intron_score[1][0][ATAC_REV] = ATAC_INTRON;
  /* "either" keeps the reference's mixed FINAL/regular values (:172-184) */
  intron_score[2][1][GTAG_FWD] = FINAL_CANONICAL_INTRON_HIGHQ;
  intron_score[2][1][GCAG_FWD] = FINAL_GCAG_INTRON;
  intron_score[2][1][ATAC_FWD] = FINAL_ATAC_INTRON;
  intron_score[2][1][GTAG_REV] = CANONICAL_INTRON_HIGHQ;
  intron_score[2][1][GCAG_REV] = FINAL_GCAG_INTRON;
  intron_score[2][1][ATAC_REV] = FINAL_ATAC_INTRON;
  intron_score[2][0][GTAG_FWD] = FINAL_CANONICAL_INTRON_HIGHQ;
  intron_score[2][0][GCAG_FWD] = GCAG_INTRON;
  intron_score[2][0][ATAC_FWD] = ATAC_INTRON;
  intron_score[2][0][GTAG_REV] = CANONICAL_INTRON_HIGHQ;
  intron_score[2][0][GCAG_REV] = GCAG_INTRON;
  intron_score[2][0][ATAC_REV] = ATAC_INTRON;
}

int
orc_intron_scores (int *out3x2x64) {
  intron_score_setup();
  memcpy(out3x2x64, intron_score, sizeof(intron_score));
  return 0;
}

/* dinucleotide codes (dynprog_genome.c:2518-2566, no genomealt: alt == ref) */
static int
left_dinucl (char left1, char left2) {
  if (left1 == 'G' && left2 == 'T') return LEFT_GT;
  if (left1 == 'G' && left2 == 'C') return LEFT_GC;
  if (left1 == 'A' && left2 == 'T') return LEFT_AT;
  if (left1 == 'C' && left2 == 'T') return LEFT_CT;
  return 0;
}

static int
right_dinucl (char right2, char right1) {
  if (right2 == 'A' && right1 == 'G') return RIGHT_AG;
  if (right2 == 'A' && right1 == 'C') return RIGHT_AC;
  if (right2 == 'G' && right1 == 'C') return RIGHT_GC;
  if (right2 == 'A' && right1 == 'T') return RIGHT_AT;
  return 0;
}

/* Splice-site positions and models of the probability arrays
   (bridge_intron_gap_site_level :2573-2660 = get_splicesite_probs :332-401).
   model: 0 donor, 1 acceptor, 2 antidonor, 3 antiacceptor.  Univcoord_T
   arithmetic is 32-bit unsigned. */
int
orc_genome_splice_sites (int glengthL, int glengthR, int goffsetL, int rev_goffsetR, unsigned int chroffset,
                         unsigned int chrhigh, int cdna_direction, int watsonp, unsigned int *posL, int *modelL,
                         unsigned int *posR, int *modelR) {
  int c;
  unsigned int leftoffset = (unsigned int) goffsetL, rightoffset = (unsigned int) rev_goffsetR;
  for (c = 0; c < glengthL; c++) {
    if (watsonp) {
      posL[c] = chroffset + leftoffset + (unsigned int) c;
      modelL[c] = cdna_direction > 0 ? 0 : 3;
    } else {
      posL[c] = chrhigh - leftoffset - (unsigned int) c + 1u;
      modelL[c] = cdna_direction > 0 ? 2 : 1;
    }
  }
  for (c = 0; c < glengthR; c++) {
    if (watsonp) {
      posR[c] = chroffset + rightoffset - (unsigned int) c + 1u;
      modelR[c] = cdna_direction > 0 ? 1 : 2;
    } else {
      posR[c] = chrhigh - rightoffset + (unsigned int) c;
      modelR[c] = cdna_direction > 0 ? 3 : 0;
    }
  }
  return 0;
}

typedef struct {
  int score, nmatches, nmismatches, nopens, nindels;
  int new_left, new_right, exonhead, introntype, dpi;
  double left_prob, right_prob;
} GGOut;

/* one diagonal cell pushed by genome_gap_simple (:3184-3272) */
static void
simple_push (PairSink *s, GGOut *o, char c1, char c1_uc, char c2, int querypos, int genomepos, int genestrand,
             int dpi) {
  if (c2 == '*') {
  } else if (c1_uc == c2) {
    o->score += MATCH; o->nmatches += 1;
    sink_push(s, querypos, genomepos, c1, DYNPROG_MATCH_COMP, c2, c2, dpi);
  } else if (consistent[genestrand][(unsigned char) c1_uc][(unsigned char) c2]) {
    o->score += MATCH; o->nmatches += 1;
    sink_push(s, querypos, genomepos, c1, AMBIGUOUS_COMP, c2, c2, dpi);
  } else {
    o->score += MISMATCH; o->nmismatches += 1;
    sink_push(s, querypos, genomepos, c1, MISMATCH_COMP, c2, c2, dpi);
  }
}

/* Known splice sites (gmap -s, get_known_splicesites dynprog_genome.c:405) for the next orc_genome_gap
   call, as flags in the engine's layout (include/gmapdp.h GMAPDP_KNOWN_SITES): the bridge's left_known
   [0, glengthL) and right_known [glengthL, +glengthR), then genome_gap_simple's left / right_known over
   rlength + 1 each.  A known site has probability 1.0 (:2577, 339) and scores KNOWN_SPLICESITE_REWARD
   in genome_gap_simple (:3118).  NULL: none (the default). */
#define KNOWN_SPLICESITE_REWARD 20
static const unsigned char *g_known = NULL;
void orc_set_known (const unsigned char *known) { g_known = known; }

/* genome_gap_simple (dynprog_genome.c:3006-3280).  Returns the number of pairs
   (reference list order) or -1 when it declines.  ks: its known-site flags (left [0, rlength],
   right after them) or NULL. */
static int
genome_gap_simple (PairSink *s, GGOut *o, const char *rsequence, const char *rsequenceuc,
                   const char *rev_rsequence, const char *rev_rsequenceuc, int rlength, const char *gL,
                   const char *revR, int roffset, int rev_roffset, int leftoffset, int rightoffset,
                   int mismatchtype, int dirclass, const double *left_probs, const double *right_probs,
                   int genestrand, int dpi, int halfp, const unsigned char *ks) {
  const int *isc = intron_score[dirclass][0];  /* assumes finalp false (:3032) */
  short (*pd)[128] = pairdistance[mismatchtype];
  int scoreL = 0, scoreR = 0, bestscore = 0, bestscoreI = 0, bestrL = -1, bestrR = -1;
  int rL, rR, r, score, scoreI, introntype, finalscore, n;

  for (rR = 1; rR < rlength; rR++) scoreR += pd[(unsigned char) rev_rsequenceuc[1 - rR]][(unsigned char) revR[1 - rR]];
  for (rL = 1, rR = rlength - 1; rL < rlength; rL++, rR--) {
    scoreL += pd[(unsigned char) rsequenceuc[rL - 1]][(unsigned char) gL[rL - 1]];
    introntype = left_dinucl(gL[rL], gL[rL + 1]) & right_dinucl(revR[-rR - 1], revR[-rR]);
    scoreI = isc[introntype];
    const int kl = (ks && ks[rL]) ? KNOWN_SPLICESITE_REWARD : 0;
    const int kr = (ks && ks[rlength + 1 + rR]) ? KNOWN_SPLICESITE_REWARD : 0;
    if ((introntype != 0 || kl > 0 || kr > 0) && (score = scoreL + kl + scoreI + kr + scoreR) >= bestscore) {
      bestscore = score;
      bestscoreI = scoreI;
      bestrL = rL;
      bestrR = rR;
      o->introntype = introntype;
    }
    scoreR -= pd[(unsigned char) rev_rsequenceuc[1 - rR]][(unsigned char) revR[1 - rR]];
  }
  finalscore = halfp ? bestscore - bestscoreI / 2 : bestscore;
  o->score = o->nmatches = o->nmismatches = 0;
  if (finalscore <= 0) return -1;
  o->left_prob = (ks && ks[bestrL]) ? 1.0 : left_probs[bestrL];  /* get_splicesite_probs (:339) */
  o->right_prob = (ks && ks[rlength + 1 + bestrR]) ? 1.0 : right_probs[bestrR];
  if (o->left_prob < 0.90 || o->right_prob < 0.90) return -1;

  for (r = 1; r <= bestrL; r++)
    simple_push(s, o, rsequence[r - 1], rsequenceuc[r - 1], gL[r - 1], roffset + r - 1, leftoffset + r - 1,
                genestrand, dpi);
  o->new_left = leftoffset + (bestrL - 1);
  o->new_right = o->exonhead = rightoffset - (bestrR - 1);
  sink_gapholder(s, 0, o->new_right - o->new_left - 1);
  for (r = bestrR; r > 0; r--)
    simple_push(s, o, rev_rsequence[1 - r], rev_rsequenceuc[1 - r], revR[1 - r], rev_roffset + 1 - r,
                rightoffset + 1 - r, genestrand, dpi);
  n = s->n < s->cap ? s->n : s->cap;
  reverse_pairs(s->buf, n);  /* pushes prepend, no List_reverse ("Already reversed") */
  return s->n;
}

/* bridge_intron_gap_site_level (dynprog_genome.c:2469-2893) with the bands of
   bridge_intron_gap (:2924-2928).  Returns finalscore. */
static int
bridge_site_level (int *bestrL, int *bestrR, int *bestcL, int *bestcR, const int *matrixL, const int *matrixR,
                   const char *gL, const char *revR, int rlength, int glengthL, int glengthR, int dirclass,
                   int finalp, int halfp, int lbandL, int ubandL, int lbandR, int ubandR, int leftoffset,
                   int rightoffset, const double *lp, const double *rp) {
  const int *isc = intron_score[dirclass][finalp ? 1 : 0];
  int *leftdi = (int *) malloc((glengthL + 1) * sizeof(int));
  int *rightdi = (int *) malloc((glengthR + 1) * sizeof(int));
  int rL, rR, cL, cR, cloL, chighL, cloR, chighR, scoreL, scoreR, scoreI, score;
  int bestscore = NEG_INFINITY_32, bestscore_with_dinucl = NEG_INFINITY_32;
  int bestrL_d = 0, bestrR_d = 0, bestcL_d = 0, bestcR_d = 0, use_dinucl_p;
  double probL, probR, bestprob_with_score = 0.0, bestprob_with_dinucl = 0.0;
#define ML(c, r) matrixL[(size_t) (c) * (size_t) (rlength + 1) + (size_t) (r)]
#define MR(c, r) matrixR[(size_t) (c) * (size_t) (rlength + 1) + (size_t) (r)]
#define CONSIDER()                                                                              \
  do {                                                                                          \
    if ((score = scoreL + scoreI + scoreR) > bestscore) {                                       \
      bestscore = score; *bestrL = rL; *bestrR = rR; *bestcL = cL; *bestcR = cR;                 \
      bestprob_with_score = probL + probR;                                                      \
    } else if (score == bestscore && probL + probR > bestprob_with_score) {                     \
      *bestrL = rL; *bestrR = rR; *bestcL = cL; *bestcR = cR;                                    \
      bestprob_with_score = probL + probR;                                                      \
    }                                                                                           \
  } while (0)

  for (cL = 0; cL < glengthL - 1; cL++) leftdi[cL] = left_dinucl(gL[cL], gL[cL + 1]);
  leftdi[glengthL - 1] = leftdi[glengthL] = 0;
  for (cR = 0; cR < glengthR - 1; cR++) rightdi[cR] = right_dinucl(revR[-cR - 1], revR[-cR]);
  rightdi[glengthR - 1] = rightdi[glengthR] = 0;

  for (rL = 1, rR = rlength - 1; rL < rlength; rL++, rR--) {
    if ((cloL = rL - lbandL) < 1) cloL = 1;
    if ((chighL = rL + ubandL) > glengthL - 1) chighL = glengthL - 1;
    if ((cloR = rR - lbandR) < 1) cloR = 1;
    if ((chighR = rR + ubandR) > glengthR - 1) chighR = glengthR - 1;

    /* A: no indels */
    cL = rL; probL = lp[cL]; scoreL = ML(cL, rL);
    cR = rR; probR = rp[cR]; scoreR = MR(cR, rR);
    scoreI = isc[leftdi[cL] & rightdi[cR]];
    CONSIDER();
    if (scoreI > 0 && probL + probR > bestprob_with_dinucl) {
      bestscore_with_dinucl = scoreL + scoreI + scoreR;
      bestcL_d = cL; bestcR_d = cR; bestrL_d = rL; bestrR_d = rR;
      bestprob_with_dinucl = probL + probR;
    }
    /* B: indel on the right */
    cL = rL; probL = lp[cL]; scoreL = ML(cL, rL);
    for (cR = cloR; cR < chighR && cR < rightoffset - leftoffset - cL; cR++) {
      probR = rp[cR];
      scoreR = MR(cR, rR);
      scoreI = isc[leftdi[cL] & rightdi[cR]];
      CONSIDER();
    }
    /* C: indel on the left */
    cR = rR; probR = rp[cR]; scoreR = MR(cR, rR);
    for (cL = cloL; cL < chighL && cL < rightoffset - leftoffset - cR; cL++) {
      probL = lp[cL];
      scoreL = ML(cL, rL);
      scoreI = isc[leftdi[cL] & rightdi[cR]];
      CONSIDER();
    }
  }
#undef CONSIDER
#undef ML
#undef MR

  if (bestprob_with_score > 2 * PROB_CEILING) use_dinucl_p = 0;
  else if (bestprob_with_dinucl == 0.0) use_dinucl_p = 0;
  else if (bestscore_with_dinucl < 0 || bestscore_with_dinucl < bestscore - 9) use_dinucl_p = 0;
  else use_dinucl_p = 1;
  if (use_dinucl_p) {
    *bestcL = bestcL_d; *bestcR = bestcR_d; *bestrL = bestrL_d; *bestrR = bestrR_d;
    bestscore = bestscore_with_dinucl;
  }
  if (bestscore >= 0 && halfp) {
    /* the reference reads leftdi/rightdi after FREEA (alloca: still valid) */
    scoreI = isc[leftdi[*bestcL] & rightdi[*bestcR]];
    bestscore = bestscore - scoreI / 2;
  }
  free(leftdi);
  free(rightdi);
  return bestscore;
}

/* bridge_intron_gap_8_site_level / _16_site_level (dynprog_genome.c:867 / :1742), reached through
   bridge_intron_gap_8_ud / _16_ud (:1388 / :2263) with the bands of Dynprog_compute_bands: the
   scan of bridge_site_level over the two triangles of each side.  B walks cR over the R lower
   triangle up to the diagonal, skips it (A covered it) and continues in the R upper triangle;
   C does the same for cL on the left.  bestscore starts at NEG_INFINITY_8/16. */
static int
bridge_ud (int *bestrL, int *bestrR, int *bestcL, int *bestcR, const int *mLu, const int *mLl, const int *mRu,
           const int *mRl, const char *gL, const char *revR, int rlength, int glengthL, int glengthR, int dirclass,
           int finalp, int halfp, int lbandL, int ubandL, int lbandR, int ubandR, int leftoffset,
           int rightoffset, const double *lp, const double *rp, int neg) {
  const int *isc = intron_score[dirclass][finalp ? 1 : 0];
  int *leftdi = (int *) malloc((glengthL + 1) * sizeof(int));
  int *rightdi = (int *) malloc((glengthR + 1) * sizeof(int));
  int rL, rR, cL, cR, cloL, chighL, cloR, chighR, scoreL, scoreR, scoreI, score;
  int bestscore = neg, bestscore_with_dinucl = neg;
  int bestrL_d = 0, bestrR_d = 0, bestcL_d = 0, bestcR_d = 0, use_dinucl_p;
  double probL, probR, bestprob_with_score = 0.0, bestprob_with_dinucl = 0.0;
#define ML(m, c, r) m[(size_t) (c) * (size_t) (rlength + 1) + (size_t) (r)]
#define CONSIDER()                                                                              \
  do {                                                                                          \
    if ((score = scoreL + scoreI + scoreR) > bestscore) {                                       \
      bestscore = score; *bestrL = rL; *bestrR = rR; *bestcL = cL; *bestcR = cR;                 \
      bestprob_with_score = probL + probR;                                                      \
    } else if (score == bestscore && probL + probR > bestprob_with_score) {                     \
      *bestrL = rL; *bestrR = rR; *bestcL = cL; *bestcR = cR;                                    \
      bestprob_with_score = probL + probR;                                                      \
    }                                                                                           \
  } while (0)

  for (cL = 0; cL < glengthL - 1; cL++) leftdi[cL] = left_dinucl(gL[cL], gL[cL + 1]);
  leftdi[glengthL - 1] = leftdi[glengthL] = 0;
  for (cR = 0; cR < glengthR - 1; cR++) rightdi[cR] = right_dinucl(revR[-cR - 1], revR[-cR]);
  rightdi[glengthR - 1] = rightdi[glengthR] = 0;

  for (rL = 1, rR = rlength - 1; rL < rlength; rL++, rR--) {
    if ((cloL = rL - lbandL) < 1) cloL = 1;
    if ((chighL = rL + ubandL) > glengthL - 1) chighL = glengthL - 1;
    if ((cloR = rR - lbandR) < 1) cloR = 1;
    if ((chighR = rR + ubandR) > glengthR - 1) chighR = glengthR - 1;

    /* A: no indels (:1082-1134) */
    cL = rL; probL = lp[cL]; scoreL = ML(mLu, cL, rL);
    cR = rR; probR = rp[cR]; scoreR = ML(mRu, cR, rR);
    scoreI = isc[leftdi[cL] & rightdi[cR]];
    CONSIDER();
    if (scoreI > 0 && probL + probR > bestprob_with_dinucl) {
      bestscore_with_dinucl = scoreL + scoreI + scoreR;
      bestcL_d = cL; bestcR_d = cR; bestrL_d = rL; bestrR_d = rR;
      bestprob_with_dinucl = probL + probR;
    }
    /* B: indel on the right (:1137-1235) */
    cL = rL; probL = lp[cL]; scoreL = ML(mLu, cL, rL);
    for (cR = cloR; cR < rR && cR < rightoffset - leftoffset - cL; cR++) {
      probR = rp[cR];
      scoreR = ML(mRl, cR, rR);
      scoreI = isc[leftdi[cL] & rightdi[cR]];
      CONSIDER();
    }
    for (cR++; cR < chighR && cR < rightoffset - leftoffset - cL; cR++) {
      probR = rp[cR];
      scoreR = ML(mRu, cR, rR);
      scoreI = isc[leftdi[cL] & rightdi[cR]];
      CONSIDER();
    }
    /* C: indel on the left (:1237-1335) */
    cR = rR; probR = rp[cR]; scoreR = ML(mRu, cR, rR);
    for (cL = cloL; cL < rL && cL < rightoffset - leftoffset - cR; cL++) {
      probL = lp[cL];
      scoreL = ML(mLl, cL, rL);
      scoreI = isc[leftdi[cL] & rightdi[cR]];
      CONSIDER();
    }
    for (cL++; cL < chighL && cL < rightoffset - leftoffset - cR; cL++) {
      probL = lp[cL];
      scoreL = ML(mLu, cL, rL);
      scoreI = isc[leftdi[cL] & rightdi[cR]];
      CONSIDER();
    }
  }
#undef CONSIDER
#undef ML

  if (bestprob_with_score > 2 * PROB_CEILING) use_dinucl_p = 0;
  else if (bestprob_with_dinucl == 0.0) use_dinucl_p = 0;
  else if (bestscore_with_dinucl < 0 || bestscore_with_dinucl < bestscore - 9) use_dinucl_p = 0;
  else use_dinucl_p = 1;
  if (use_dinucl_p) {
    *bestcL = bestcL_d; *bestcR = bestcR_d; *bestrL = bestrL_d; *bestrR = bestrR_d;
    bestscore = bestscore_with_dinucl;
  }
  if (bestscore >= 0 && halfp) {
    scoreI = isc[leftdi[*bestcL] & rightdi[*bestcR]];
    bestscore = bestscore - scoreI / 2;
  }
  free(leftdi);
  free(rightdi);
  return bestscore;
}

/* Pair_maxnegscore (pair.c:8528) over pairs in list order */
static int
maxnegscore (const OrcPair *p, int n) {
  int maxneg = 0, prevhigh = 0, score = 0, i = 0;
  while (i < n) {
    if (p[i].gapp) {
      i++;
    } else if (p[i].comp == MISMATCH_COMP) {
      score += MISMATCH;
      if (score - prevhigh < maxneg) maxneg = score - prevhigh;
      i++;
    } else if (p[i].comp == INDEL_COMP) {
      score += QOPEN + QINDEL;
      i++;
      while (i < n && p[i].comp == INDEL_COMP) { score += QINDEL; i++; }
      if (score - prevhigh < maxneg) maxneg = score - prevhigh;
    } else {
      score += MATCH;
      if (score > prevhigh) prevhigh = score;
      i++;
    }
  }
  return maxneg;
}

static void
gg_scalars (const GGOut *o, int *scalars, double *dscalars) {
  scalars[0] = o->dpi; scalars[1] = o->score; scalars[2] = o->nmatches; scalars[3] = o->nmismatches;
  scalars[4] = o->nopens; scalars[5] = o->nindels; scalars[6] = o->new_left; scalars[7] = o->new_right;
  scalars[8] = o->exonhead; scalars[9] = o->introntype;
  dscalars[0] = o->left_prob; dscalars[1] = o->right_prob;
}

/* The tail of Dynprog_genome_gap after the second traceback (:3872-3896): counters, NULL when
   only the gap holder was pushed, Pair_maxnegscore rejection.  Returns the pair count or -1. */
static int
gg_finish (PairSink *sink, const Tally *t, GGOut *o, OrcPair *out, int max_pairs, int dynprogindex) {
  int n, i;
  o->score = t->score; o->nmatches = t->nmatches; o->nmismatches = t->nmismatches;
  o->nopens = t->nopens; o->nindels = t->nindels;
  o->dpi = dynprogindex + (dynprogindex > 0 ? +1 : -1);
  n = sink->n;
  if (n == 1) {
    n = -1;  /* only the gap holder: NULL (:3877) */
  } else {
    /* before the final List_reverse the list is reverse(TL), G, TR in its own order:
       the reverse of what is returned */
    OrcPair *tmp = (OrcPair *) malloc((size_t) n * sizeof(OrcPair));
    int m = n < max_pairs ? n : max_pairs;
    for (i = 0; i < m; i++) tmp[i] = out[m - 1 - i];
    if (maxnegscore(tmp, m) < -10) {
      o->score = -100;
      n = -1;
    }
    free(tmp);
  }
  return n;
}

/* flags: 1 watsonp, 2 jump_late_p, 8 halfp, 16 finalp. */
int
orc_genome_gap (const char *rsequence, const char *rsequenceuc, int rlength, int glengthL, int glengthR,
                int roffset, int goffsetL, int rev_goffsetR, unsigned int chroffset, unsigned int chrhigh,
                int cdna_direction, int flags, int genestrand, int extraband_paired, double defect_rate,
                int maxpeelback, int dynprogindex, const double *left_probs, const double *right_probs,
                int *scalars, double *dscalars, OrcPair *out, int max_pairs) {
  const int watsonp = flags & 1, jump_late_p = (flags & 2) ? 1 : 0, halfp = (flags & 8) ? 1 : 0;
  const int finalp = (flags & 16) ? 1 : 0;
  const int dirclass = cdna_direction > 0 ? 0 : (cdna_direction < 0 ? 1 : 2);
  int mismatchtype, open, extend, lbandL, ubandL, lbandR, ubandR, finalscore, n, nR;
  int bestrL = -1, bestrR = 0, bestcL = 0, bestcR = 0;
  int rev_roffset;
  char *gL, *gLa, *gR, *gRa;
  const char *revR, *rev_rsequence, *rev_rsequenceuc;
  int *matrixL, *matrixR;
  signed char *dirsL, *dirsR;
  PairSink sink = {out, 0, max_pairs};
  Tally t = {0, 0, 0, 0, 0};
  GGOut o;

  o.score = ORC_UNSET;
  o.nmatches = o.nmismatches = o.nopens = o.nindels = 0;
  o.new_left = o.new_right = o.exonhead = ORC_UNSET;
  o.introntype = 0;
  o.left_prob = o.right_prob = 0.0;
  o.dpi = dynprogindex;
  if (rlength <= 1) {
    o.score = NEG_INFINITY_32;
    gg_scalars(&o, scalars, dscalars);
    return -1;
  }
  if (defect_rate < DEFECT_HIGHQ) mismatchtype = HIGHQ;
  else if (defect_rate < DEFECT_MEDQ) mismatchtype = MEDQ;
  else mismatchtype = LOWQ;
  if (g_user_dynprog_p) { open = g_user_open; extend = g_user_extend; }
  else if (defect_rate < DEFECT_HIGHQ) {
    if (rlength > maxpeelback * 4) { open = SINGLE_OPEN_HIGHQ; extend = SINGLE_EXTEND_HIGHQ; }
    else { open = PAIRED_OPEN_HIGHQ; extend = PAIRED_EXTEND_HIGHQ; }
  } else if (defect_rate < DEFECT_MEDQ) {
    if (rlength > maxpeelback * 4) { open = SINGLE_OPEN_MEDQ; extend = SINGLE_EXTEND_MEDQ; }
    else { open = PAIRED_OPEN_MEDQ; extend = PAIRED_EXTEND_MEDQ; }
  } else {
    if (rlength > maxpeelback * 4) { open = SINGLE_OPEN_LOWQ; extend = SINGLE_EXTEND_LOWQ; }
    else { open = PAIRED_OPEN_LOWQ; extend = PAIRED_EXTEND_LOWQ; }
  }
  if (rlength > ORC_MAX_RLENGTH || glengthL > ORC_MAX_GLENGTH || glengthR > ORC_MAX_GLENGTH) {
    o.new_left = goffsetL - 1;
    o.new_right = rev_goffsetR + 1;
    o.exonhead = roffset + rlength - 1;
    o.dpi = dynprogindex + (dynprogindex > 0 ? +1 : -1);
    o.score = NEG_INFINITY_32;
    gg_scalars(&o, scalars, dscalars);
    return -1;
  }
  rev_rsequence = rsequence + rlength - 1;
  rev_rsequenceuc = rsequenceuc + rlength - 1;
  rev_roffset = roffset + rlength - 1;
  gL = (char *) malloc(glengthL + 1); gLa = (char *) malloc(glengthL + 1);
  gR = (char *) malloc(glengthR + 1); gRa = (char *) malloc(glengthR + 1);
  if (watsonp) {
    orc_get_segment(1, chroffset + (unsigned int) goffsetL, glengthL, chrhigh, 0, gL, gLa);
    orc_get_segment(0, chroffset + (unsigned int) rev_goffsetR + 1u, glengthR, chroffset, 0, gR, gRa);
  } else {
    orc_get_segment(0, chrhigh - (unsigned int) goffsetL + 1u, glengthL, chroffset, 1, gL, gLa);
    orc_get_segment(1, chrhigh - (unsigned int) rev_goffsetR, glengthR, chrhigh, 1, gR, gRa);
  }
  if (gL[0] == '\0' || gR[0] == '\0') {
    o.score = NEG_INFINITY_32;
    free(gL); free(gLa); free(gR); free(gRa);
    gg_scalars(&o, scalars, dscalars);
    return -1;
  }
  revR = gR + glengthR - 1;

  if (!finalp && defect_rate < DEFECT_MEDQ) {
    n = genome_gap_simple(&sink, &o, rsequence, rsequenceuc, rev_rsequence, rev_rsequenceuc, rlength, gL, revR,
                          roffset, rev_roffset, goffsetL, rev_goffsetR, mismatchtype, dirclass, left_probs,
                          right_probs, genestrand, dynprogindex, halfp,
                          g_known ? g_known + glengthL + glengthR : NULL);
    if (n >= 0) {
      o.dpi = dynprogindex + (dynprogindex > 0 ? +1 : -1);
      free(gL); free(gLa); free(gR); free(gRa);
      gg_scalars(&o, scalars, dscalars);
      return n;
    }
    sink.n = 0;
  }

  /* known sites: probability 1.0 in the bridge of either build (dynprog_genome.c:2577-2652, 978-1053) */
  double *lpk = NULL, *rpk = NULL;
  if (g_known) {
    int c;
    lpk = (double *) malloc((glengthL + 1) * sizeof(double));
    rpk = (double *) malloc((glengthR + 1) * sizeof(double));
    for (c = 0; c < glengthL; c++) lpk[c] = g_known[c] ? 1.0 : left_probs[c];
    for (c = 0; c < glengthR; c++) rpk[c] = g_known[glengthL + c] ? 1.0 : right_probs[c];
    left_probs = lpk;
    right_probs = rpk;
  }
  if (g_simd) {
    /* dynprog_genome.c:3501-3795: 8-bit triangles when rlength or both glengths are below use8p_size */
    int bits = (rlength < use8p_size[mismatchtype] ||
                (glengthL < use8p_size[mismatchtype] && glengthR < use8p_size[mismatchtype])) ? 8 : 16;
    size_t pl = (size_t) (glengthL + 1) * (rlength + 1), pr = (size_t) (glengthR + 1) * (rlength + 1);
    int *mL = (int *) malloc(2 * pl * sizeof(int)), *mR = (int *) malloc(2 * pr * sizeof(int));
    signed char *dL = (signed char *) malloc(6 * pl), *dR = (signed char *) malloc(6 * pr);
    compute_bands(&lbandL, &ubandL, rlength, glengthL, extraband_paired, 1);
    simd_fill_ud(bits, 1, rsequence, gL, gL, rlength, glengthL, mismatchtype, open, extend, ubandL, jump_late_p, 0,
                 mL, dL);
    simd_fill_ud(bits, 0, rsequence, gL, gL, rlength, glengthL, mismatchtype, open, extend, lbandL, jump_late_p, 0,
                 mL + pl, dL + 3 * pl);
    compute_bands(&lbandR, &ubandR, rlength, glengthR, extraband_paired, 1);
    simd_fill_ud(bits, 1, rev_rsequence, revR, revR, rlength, glengthR, mismatchtype, open, extend, ubandR,
                 !jump_late_p, 1, mR, dR);
    simd_fill_ud(bits, 0, rev_rsequence, revR, revR, rlength, glengthR, mismatchtype, open, extend, lbandR,
                 !jump_late_p, 1, mR + pr, dR + 3 * pr);
    finalscore = bridge_ud(&bestrL, &bestrR, &bestcL, &bestcR, mL, mL + pl, mR, mR + pr, gL, revR, rlength,
                           glengthL, glengthR, dirclass, finalp, halfp, lbandL, ubandL, lbandR, ubandR, goffsetL,
                           rev_goffsetR, left_probs, right_probs, bits == 8 ? -128 : -32768);
    if (finalscore < 0) {
      o.score = -100;
      n = -1;
    } else {
      int upR = bestcR >= bestrR, upL = bestcL >= bestrL;
      o.left_prob = left_probs[bestcL];
      o.right_prob = right_probs[bestcR];
      o.new_left = goffsetL + (bestcL - 1);
      o.new_right = rev_goffsetR - (bestcR - 1);
      o.exonhead = rev_roffset - (bestrR - 1);
      traceback_mode(&sink, &t, upR ? dR : dR + 3 * pr, rlength, glengthR, bestrR, bestcR, rev_rsequence,
                     rev_rsequenceuc, revR, revR, rev_roffset, rev_goffsetR, /*revp*/1, chroffset, chrhigh, watsonp,
                     genestrand, dynprogindex, upR ? 1 : 2);
      nR = sink.n < max_pairs ? sink.n : max_pairs;
      reverse_pairs(out, nR);
      sink_gapholder(&sink, (rev_roffset - bestrR) - (roffset + bestrL) + 1, o.new_right - o.new_left - 1);
      traceback_mode(&sink, &t, upL ? dL : dL + 3 * pl, rlength, glengthL, bestrL, bestcL, rsequence, rsequenceuc,
                     gL, gL, roffset, goffsetL, /*revp*/0, chroffset, chrhigh, watsonp, genestrand, dynprogindex,
                     upL ? 1 : 2);
      n = gg_finish(&sink, &t, &o, out, max_pairs, dynprogindex);
    }
    free(mL); free(mR); free(dL); free(dR);
    free(lpk); free(rpk);
    free(gL); free(gLa); free(gR); free(gRa);
    gg_scalars(&o, scalars, dscalars);
    return n;
  }

  compute_bands(&lbandL, &ubandL, rlength, glengthL, extraband_paired, 1);
  matrixL = (int *) malloc((size_t) (glengthL + 1) * (rlength + 1) * sizeof(int));
  dirsL = (signed char *) malloc((size_t) 3 * (glengthL + 1) * (rlength + 1));
  orc_standard_fill(rsequence, gL, gL, rlength, glengthL, mismatchtype, open, extend, lbandL, ubandL,
                    jump_late_p, /*revp*/0, NEG_INFINITY_32, 1, 1, matrixL, dirsL);
  compute_bands(&lbandR, &ubandR, rlength, glengthR, extraband_paired, 1);
  matrixR = (int *) malloc((size_t) (glengthR + 1) * (rlength + 1) * sizeof(int));
  dirsR = (signed char *) malloc((size_t) 3 * (glengthR + 1) * (rlength + 1));
  /* the reference passes lbandL here (dynprog_genome.c:3813) */
  orc_standard_fill(rev_rsequence, revR, revR, rlength, glengthR, mismatchtype, open, extend, lbandL, ubandR,
                    !jump_late_p, /*revp*/1, NEG_INFINITY_32, 1, 1, matrixR, dirsR);

  /* bridge_intron_gap's own bands (:2924-2928) */
  finalscore = bridge_site_level(&bestrL, &bestrR, &bestcL, &bestcR, matrixL, matrixR, gL, revR, rlength,
                                 glengthL, glengthR, dirclass, finalp, halfp,
                                 extraband_paired, glengthL - rlength + extraband_paired,
                                 extraband_paired, glengthR - rlength + extraband_paired,
                                 goffsetL, rev_goffsetR, left_probs, right_probs);
  if (finalscore < 0) {
    o.score = -100;
    n = -1;
  } else {
    o.left_prob = left_probs[bestcL];
    o.right_prob = right_probs[bestcR];
    o.new_left = goffsetL + (bestcL - 1);
    o.new_right = rev_goffsetR - (bestcR - 1);
    o.exonhead = rev_roffset - (bestrR - 1);
    traceback_std(&sink, &t, dirsR, rlength, glengthR, bestrR, bestcR, rev_rsequence, rev_rsequenceuc, revR, revR,
                  rev_roffset, rev_goffsetR, /*revp*/1, chroffset, chrhigh, watsonp, genestrand, dynprogindex);
    nR = sink.n < max_pairs ? sink.n : max_pairs;
    reverse_pairs(out, nR);  /* List_reverse (:3848) */
    sink_gapholder(&sink, (rev_roffset - bestrR) - (roffset + bestrL) + 1, o.new_right - o.new_left - 1);
    traceback_std(&sink, &t, dirsL, rlength, glengthL, bestrL, bestcL, rsequence, rsequenceuc, gL, gL,
                  roffset, goffsetL, /*revp*/0, chroffset, chrhigh, watsonp, genestrand, dynprogindex);
    n = gg_finish(&sink, &t, &o, out, max_pairs, dynprogindex);
  }
  /* returned list: List_reverse of [reverse(TL) G TR] = reverse(TR) G TL, which is the sink order */
  free(matrixL); free(dirsL); free(matrixR); free(dirsR);
  free(gL); free(gLa); free(gR); free(gRa);
  free(lpk); free(rpk);
  gg_scalars(&o, scalars, dscalars);
  return n;
}

/* ---------------------------------------------------------------------------
 * Dynprog_cdna_gap (dynprog_cdna.c:787-1300): a cDNA insertion.  L fills the
 * query piece rsequenceL forward against gsequence, R the piece ending at
 * rev_rsequenceR backwards against rev_gsequence (the same genome interval);
 * the bridge picks the split (cL, cR, rL, rR) allowing a genomic insertion
 * (pen = 0 for cR = glength - cL, else open + extend per further column).
 * Penalties are CDNA_OPEN/EXTEND (-10/-7) for every defect rate; user
 * penalties are not consulted.  Both builds: nosimd (Dynprog_standard,
 * bridge_cdna_gap :652 with its own bands, the R fill called with lbandL)
 * and SIMD (the triangles, bridge_cdna_gap_8/16_ud :124/387 with the fill
 * bands, upper cells for r < c and lower cells for r >= c).
 * ------------------------------------------------------------------------- */
#define CDNA_OPEN -10
#define CDNA_EXTEND -7
#define INSERT_PAIRS 9
#define SHORTGAP_COMP '~'

/* The candidate scan shared by both bridges: for cL, cR (descending), rL, rR the score
   cell(L, cL, rL) + cell(R, cR, rR) + pen, > (jump early) or >= (jump late). */
typedef int (*CellFn) (const int *mu, const int *ml, int rlength, int c, int r);
static int cell_std (const int *mu, const int *ml, int rlength, int c, int r) {
  (void) ml;
  return mu[(size_t) c * (rlength + 1) + r];
}
static int cell_ud (const int *mu, const int *ml, int rlength, int c, int r) {
  return (r < c ? mu : ml)[(size_t) c * (rlength + 1) + r];   /* upper[c][r] for r < c, else lower[r][c] */
}

static int
bridge_cdna (int *bestcL, int *bestcR, int *bestrL, int *bestrR, CellFn cell, const int *mLu, const int *mLl,
             const int *mRu, const int *mRl, int glength, int rlengthL, int rlengthR, int lbandL, int ubandL,
             int lbandR, int ubandR, int open, int extend, int leftoffset, int rightoffset, int late, int neg) {
  int bestscore = neg, score, scoreL, scoreR, pen, rL, rR, cL, cR, rloL, rhighL, rloR, rhighR;
  for (cL = 1; cL < glength; cL++) {
    for (cR = glength - cL, pen = 0; cR >= 0; cR--, pen += extend) {
      if ((rloL = cL - ubandL) < 1) rloL = 1;
      if ((rhighL = cL + lbandL) > rlengthL - 1) rhighL = rlengthL - 1;
      if ((rloR = cR - ubandR) < 1) rloR = 1;
      if ((rhighR = cR + lbandR) > rlengthR - 1) rhighR = rlengthR - 1;
      for (rL = rloL; rL <= rhighL; rL++) {
        scoreL = cell(mLu, mLl, rlengthL, cL, rL);
        for (rR = rloR; rR <= rhighR && rR < rightoffset - leftoffset - rL; rR++) {
          scoreR = cell(mRu, mRl, rlengthR, cR, rR);
          if (prefer(score = scoreL + scoreR + pen, bestscore, late)) {
            bestscore = score;
            *bestcL = cL; *bestcR = cR; *bestrL = rL; *bestrR = rR;
          }
        }
      }
      pen = open - extend;
    }
  }
  return bestscore;
}

/* Domain: rlengthL == rlengthR >= glength >= 2 -- what stage3.c passes (both lengths
   queryjump = genomejump + extramaterial_paired, stage3.c:9275).  There the nosimd bridge's own
   bands equal the fills' (and lbandL = lbandR), so every cell it reads was computed; outside it
   the reference reads cells no fill wrote.  Returns -3 outside the domain. */
int
orc_cdna_gap (const char *qbuf, const char *qucbuf, int qposL, int qposR, int rlengthL, int rlengthR, int glength,
              int roffsetL, int rev_roffsetR, int goffset, unsigned int chroffset, unsigned int chrhigh,
              int watsonp, int genestrand, int jump_late_p, int extraband_paired, double defect_rate,
              int dynprogindex, int *scalars, OrcPair *out, int max_pairs) {
  const char *rsequenceL = qbuf + qposL, *rsequence_ucL = qucbuf + qposL;
  const char *rev_rsequenceR = qbuf + qposR, *rev_rsequence_ucR = qucbuf + qposR;
  int mismatchtype, lbandL, ubandL, lbandR, ubandR, rev_goffset, bestrL = 0, bestrR = 0, bestcL = 0, bestcR = 0;
  int queryjump, genomejump, k, n, bits = 32;
  char *gs, *gsa, *rgs, *rgsa, c2, c2_alt;
  const char *revg;
  size_t pl, pr;
  int *mL, *mR;
  signed char *dL, *dR;
  PairSink sink = {out, 0, max_pairs};
  Tally t = {0, 0, 0, 0, 0};

  scalars[0] = dynprogindex; scalars[1] = ORC_UNSET; scalars[2] = 0;
  if (glength <= 1) return -1;
  if (defect_rate < DEFECT_HIGHQ) mismatchtype = HIGHQ;
  else if (defect_rate < DEFECT_MEDQ) mismatchtype = MEDQ;
  else mismatchtype = LOWQ;
  if (glength > ORC_MAX_GLENGTH || rlengthR > ORC_MAX_RLENGTH || rlengthL > ORC_MAX_RLENGTH) {
    scalars[0] = dynprogindex + (dynprogindex > 0 ? +1 : -1);
    return -1;
  }
  if (rlengthL != rlengthR || rlengthL < glength) return -3;
  rev_goffset = goffset + glength - 1;
  gs = (char *) malloc(glength + 1); gsa = (char *) malloc(glength + 1);
  rgs = (char *) malloc(glength + 1); rgsa = (char *) malloc(glength + 1);
  if (watsonp) {
    orc_get_segment(0, chroffset + (unsigned int) rev_goffset + 1u, glength, chroffset, 0, rgs, rgsa);
    orc_get_segment(1, chroffset + (unsigned int) goffset, glength, chrhigh, 0, gs, gsa);
  } else {
    orc_get_segment(1, chrhigh - (unsigned int) rev_goffset, glength, chrhigh, 1, rgs, rgsa);
    orc_get_segment(0, chrhigh - (unsigned int) goffset + 1u, glength, chroffset, 1, gs, gsa);
  }
  if (gs[0] == '\0' || rgs[0] == '\0') {
    free(gs); free(gsa); free(rgs); free(rgsa);
    return -1;
  }
  revg = rgs + glength - 1;
  pl = (size_t) (glength + 1) * (rlengthL + 1);
  pr = (size_t) (glength + 1) * (rlengthR + 1);
  mL = (int *) malloc(2 * pl * sizeof(int)); mR = (int *) malloc(2 * pr * sizeof(int));
  dL = (signed char *) malloc(6 * pl); dR = (signed char *) malloc(6 * pr);
  compute_bands(&lbandL, &ubandL, rlengthL, glength, extraband_paired, 1);
  compute_bands(&lbandR, &ubandR, rlengthR, glength, extraband_paired, 1);
  if (g_simd) {
    /* :898-904: 8-bit when glength is below use8p_size, or rlengthL is and rlengthR is not above it */
    const int u = use8p_size[mismatchtype];
    bits = (glength < u || (rlengthL < u && rlengthR <= u)) ? 8 : 16;
    simd_fill_ud(bits, 1, rsequenceL, gs, gs, rlengthL, glength, mismatchtype, CDNA_OPEN, CDNA_EXTEND, ubandL,
                 jump_late_p, 0, mL, dL);
    simd_fill_ud(bits, 0, rsequenceL, gs, gs, rlengthL, glength, mismatchtype, CDNA_OPEN, CDNA_EXTEND, lbandL,
                 jump_late_p, 0, mL + pl, dL + 3 * pl);
    simd_fill_ud(bits, 1, rev_rsequenceR, revg, revg, rlengthR, glength, mismatchtype, CDNA_OPEN, CDNA_EXTEND,
                 ubandR, !jump_late_p, 1, mR, dR);
    simd_fill_ud(bits, 0, rev_rsequenceR, revg, revg, rlengthR, glength, mismatchtype, CDNA_OPEN, CDNA_EXTEND,
                 lbandR, !jump_late_p, 1, mR + pr, dR + 3 * pr);
    bridge_cdna(&bestcL, &bestcR, &bestrL, &bestrR, cell_ud, mL, mL + pl, mR, mR + pr, glength, rlengthL, rlengthR,
                lbandL, ubandL, lbandR, ubandR, CDNA_OPEN, CDNA_EXTEND, roffsetL, rev_roffsetR, jump_late_p,
                bits == 8 ? -128 : -32768);
  } else {
    orc_standard_fill(rsequenceL, gs, gs, rlengthL, glength, mismatchtype, CDNA_OPEN, CDNA_EXTEND, lbandL, ubandL,
                      jump_late_p, 0, NEG_INFINITY_32, 1, 1, mL, dL);
    /* the reference passes lbandL to the R fill (dynprog_cdna.c:1227) */
    orc_standard_fill(rev_rsequenceR, revg, revg, rlengthR, glength, mismatchtype, CDNA_OPEN, CDNA_EXTEND, lbandL,
                      ubandR, !jump_late_p, 1, NEG_INFINITY_32, 1, 1, mR, dR);
    /* bridge_cdna_gap's own bands (:667-670) */
    bridge_cdna(&bestcL, &bestcR, &bestrL, &bestrR, cell_std, mL, NULL, mR, NULL, glength, rlengthL, rlengthR,
                rlengthL - glength + extraband_paired, extraband_paired, rlengthR - glength + extraband_paired,
                extraband_paired, CDNA_OPEN, CDNA_EXTEND, roffsetL, rev_roffsetR, jump_late_p, NEG_INFINITY_32);
  }
  /* traceback R (upper/lower by bestc >= bestr in the SIMD build), List_reverse */
  if (g_simd) {
    int up = bestcR >= bestrR;
    traceback_mode(&sink, &t, up ? dR : dR + 3 * pr, rlengthR, glength, bestrR, bestcR, rev_rsequenceR,
                   rev_rsequence_ucR, revg, revg, rev_roffsetR, rev_goffset, 1, chroffset, chrhigh, watsonp,
                   genestrand, dynprogindex, up ? 1 : 2);
  } else {
    traceback_std(&sink, &t, dR, rlengthR, glength, bestrR, bestcR, rev_rsequenceR, rev_rsequence_ucR, revg, revg,
                  rev_roffsetR, rev_goffset, 1, chroffset, chrhigh, watsonp, genestrand, dynprogindex);
  }
  n = sink.n < max_pairs ? sink.n : max_pairs;
  reverse_pairs(out, n);
  queryjump = (rev_roffsetR - bestrR) - (roffsetL + bestrL) + 1;
  genomejump = (rev_goffset - bestcR) - (goffset + bestcL) + 1;
  if (queryjump == INSERT_PAIRS && genomejump == INSERT_PAIRS) {
    for (k = rev_roffsetR - bestrR; k >= roffsetL + bestrL; k--)
      sink_push(&sink, k, rev_goffset - bestcR + 1, rsequenceL[k - roffsetL], SHORTGAP_COMP, ' ', ' ', dynprogindex);
    for (k = rev_goffset - bestcR; k >= goffset + bestcL; k--) {
      c2 = get_genomic_nt(&c2_alt, k, chroffset, chrhigh, watsonp);
      sink_push(&sink, roffsetL + bestrL, k, ' ', SHORTGAP_COMP, c2, c2_alt, dynprogindex);
    }
  } else {
    sink_gapholder(&sink, queryjump, genomejump);
    scalars[2] = 1;
  }
  if (g_simd) {
    int up = bestcL >= bestrL;
    traceback_mode(&sink, &t, up ? dL : dL + 3 * pl, rlengthL, glength, bestrL, bestcL, rsequenceL, rsequence_ucL,
                   gs, gs, roffsetL, goffset, 0, chroffset, chrhigh, watsonp, genestrand, dynprogindex, up ? 1 : 2);
  } else {
    traceback_std(&sink, &t, dL, rlengthL, glength, bestrL, bestcL, rsequenceL, rsequence_ucL, gs, gs, roffsetL,
                  goffset, 0, chroffset, chrhigh, watsonp, genestrand, dynprogindex);
  }
  scalars[0] = dynprogindex + (dynprogindex > 0 ? +1 : -1);
  scalars[1] = t.score;
  n = sink.n;
  free(mL); free(mR); free(dL); free(dR); free(gs); free(gsa); free(rgs); free(rgsa);
  if (n == 1) return -1;  /* only the gap added (:1284) */
  /* returned: List_reverse of [reverse(TL) reverse(I) TR] = reverse(TR) I TL, the sink order */
  return n;
}
