// vbfm_host.cpp -- host side of the reference's CLI path, exported through include/vbfm.h:
//   * vbfm_load_data        Data::load (src/libfm/src/Data.h:106-283): libfm text with the
//                           reference's sscanf semantics, or the binary .x/.xt/.y triple
//                           (src/util/fmatrix.h:46-52,66-82; src/util/matrix.h:296-312)
//   * vbfm_init_params_host the reference's initial draws (glibc rand() after srand(seed),
//                           Leva normals: src/util/random.h:150-176) in its exact order, on
//                           a private copy of that generator (vbfm_rng.h).
// Plain C++; built with -ffp-contract=off like the reference's x86-64 build (no FMA).
#include "../../include/vbfm.h"
#include "vbfm_rng.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_host_err;

bool file_exists(const std::string &f)
{
	FILE *fp = fopen(f.c_str(), "rb");
	if (!fp) return false;
	fclose(fp);
	return true;
}

// ---- libfm text (Data.h:185-278) -----------------------------------------------------------
// The reference parses each line with sscanf("%f%n") and then sscanf("%d:%f%n") pairs. This
// parser keeps those semantics byte for byte without calling sscanf per line: strtol base 10
// for %d (what glibc's scanf converts with), a literal ':', the whitespace sscanf skips
// before a conversion (space, \t, \v, \f, \r; a line never holds \n), and the reference's
// checks: leading spaces / tabs, empty and '#' lines skipped, after the pairs only spaces /
// tabs and an optional '#' comment. Lines end at '\n' or at the buffer's NUL.
inline bool scan_ws(char c) { return c == ' ' || c == '\t' || c == '\v' || c == '\f' || c == '\r'; }

// %f: glibc's scanf and strtof agree on plain decimal numbers ([+-]digits[.digits][e[+-]digits])
// but not on malformed or exotic ones ("1e", "0x", "infin", "nan(1)"): a token that strtof
// does not consume whole, or that holds other characters than [0-9.eE+-], is converted by
// sscanf itself from a NUL-terminated copy. Every character %f can consume is in
// [0-9A-Za-z.+-()], so the copy holds all sscanf could read. Returns the end, or nullptr.
const char *scan_float(const char *q, const char *eol, float *v)
{
	const char *t = q;
	bool plain = true;
	while (t < eol) {
		const char c = *t;
		const bool dec = (c >= '0' && c <= '9') || c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-';
		if (!dec && !((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '(' || c == ')')) break;
		plain &= dec;
		t++;
	}
	if (t == q) return nullptr;
	if (plain) {
		char *end = nullptr;
		const float x = strtof(q, &end);
		if (end == t) { *v = x; return end; }
	}
	char tok[512];
	const size_t len = std::min<size_t>(t - q, sizeof(tok) - 1);
	memcpy(tok, q, len);
	tok[len] = 0;
	int n = 0;
	if (sscanf(tok, "%f%n", v, &n) < 1) return nullptr;
	return q + n;
}

struct LineError { size_t pos = SIZE_MAX; std::string msg; };

// 1: a row, 0: skipped line, -1: parse error (*at = the offending character)
int parse_line(const char *p, const char *eol, float *target, std::vector<vbfm_entry> &ents, int *maxf, char *at)
{
	while (p < eol && (*p == ' ' || *p == '\t')) p++;           // Data.h:196
	if (p == eol || *p == '#') return 0;                        // :197
	const char *q = p;
	while (q < eol && scan_ws(*q)) q++;
	float y = 0.f;
	const char *end = scan_float(q, eol, &y);
	if (!end) { *at = *p; return -1; }                          // sscanf("%f") < 1
	*target = y;
	p = end;
	for (;;) {                                                  // sscanf("%d:%f%n") >= 2
		q = p;
		while (q < eol && scan_ws(*q)) q++;
		if (q == eol) break;
		char *e1 = nullptr;
		const long fid = strtol(q, &e1, 10);
		if (e1 == q || *e1 != ':') break;
		const char *r = e1 + 1;
		while (r < eol && scan_ws(*r)) r++;
		float x = 0.f;
		end = scan_float(r, eol, &x);
		if (!end) break;
		const int id = (int)fid;
		if (id < 0) { *at = *q; return -1; }
		if (id > *maxf) *maxf = id;
		ents.push_back(vbfm_entry{(uint32_t)id, x});
		p = end;
	}
	while (p < eol && (*p == ' ' || *p == '\t')) p++;           // :207
	if (p < eol && *p != '#') { *at = *p; return -1; }          // :208-210
	return 1;
}

template <class T> T *xalloc(size_t n) { return (T *)malloc((n ? n : 1) * sizeof(T)); }

int num_threads()
{
	const char *env = getenv("VBFM_LOADER_THREADS");
	if (env && atoi(env) > 0) return atoi(env);
	const unsigned hw = std::thread::hardware_concurrency();
	return (int)std::max(1u, std::min(hw ? hw : 1u, 16u));      // the GPU box's CPU share is 16
}

// run fn(t) on T threads (t = 0 on the caller)
template <class F> void parallel(int T, F &&fn)
{
	std::vector<std::thread> th;
	for (int t = 1; t < T; t++) th.emplace_back(fn, t);
	fn(0);
	for (auto &x : th) x.join();
}

// Data::create_data_t (Data.h:457-509): stable counting transpose, ascending rows per column.
// Parallel over row ranges: per-range column counts give every range its own slot in every
// column, so each range scatters its rows in order and the result is the sequential one.
void transpose(vbfm_host_data *d)
{
	const uint32_t nf = d->num_feature, n = d->num_rows;
	d->col_ptr = xalloc<uint64_t>((size_t)nf + 1);
	d->col_ent = xalloc<vbfm_entry>(d->nnz);
	int T = num_threads();
	if ((uint64_t)T * nf > (uint64_t)1 << 31 || d->nnz < ((uint64_t)1 << 20)) T = 1;   // count-table memory / tiny sets
	std::vector<uint32_t> lo(T + 1);
	for (int t = 0; t <= T; t++) lo[t] = (uint32_t)((uint64_t)n * t / T);
	std::vector<uint64_t> cnt((size_t)T * nf, 0);
	parallel(T, [&](int t) {
		uint64_t *c = cnt.data() + (size_t)t * nf;
		for (uint64_t j = d->row_ptr[lo[t]]; j < d->row_ptr[lo[t + 1]]; j++) c[d->row_ent[j].id]++;
	});
	uint64_t acc = 0;
	for (uint32_t i = 0; i < nf; i++) {
		d->col_ptr[i] = acc;
		for (int t = 0; t < T; t++) {
			const uint64_t v = cnt[(size_t)t * nf + i];
			cnt[(size_t)t * nf + i] = acc;
			acc += v;
		}
	}
	d->col_ptr[nf] = acc;
	parallel(T, [&](int t) {
		uint64_t *c = cnt.data() + (size_t)t * nf;
		for (uint32_t r = lo[t]; r < lo[t + 1]; r++)
			for (uint64_t j = d->row_ptr[r]; j < d->row_ptr[r + 1]; j++) {
				const vbfm_entry &e = d->row_ent[j];
				d->col_ent[c[e.id]++] = vbfm_entry{r, e.value};
			}
	});
}

// the file in chunks of whole lines, parsed in parallel, concatenated in file order
int load_text(const char *fn, vbfm_host_data *out)
{
	FILE *fp = fopen(fn, "rb");
	if (!fp) { g_host_err = std::string("unable to open ") + fn; return -1; }
	fseeko(fp, 0, SEEK_END);
	const size_t size = (size_t)ftello(fp);
	fseeko(fp, 0, SEEK_SET);
	char *buf = xalloc<char>(size + 1);
	if (size && fread(buf, 1, size, fp) != size) {
		free(buf); fclose(fp);
		g_host_err = std::string("unable to read ") + fn;
		return -1;
	}
	fclose(fp);
	buf[size] = 0;
	const int T = size < ((size_t)1 << 20) ? 1 : num_threads();
	std::vector<size_t> cut(T + 1, size);
	cut[0] = 0;
	for (int t = 1; t < T; t++) {
		size_t c = std::max(cut[t - 1], size * t / T);
		while (c < size && c > 0 && buf[c - 1] != '\n') c++;
		cut[t] = c;
	}
	struct Part {
		std::vector<vbfm_entry> ents;
		std::vector<float> target;
		std::vector<uint32_t> len;
		int maxf = -1;
		bool has_feature = false;
		bool has_nan = false;   // a NaN target: the fold below restarts there
		float mn = 3.40282347e+38f, mx = -3.40282347e+38f;
		LineError err;
	};
	std::vector<Part> part(T);
	parallel(T, [&](int t) {
		Part &P = part[t];
		const char *p = buf + cut[t], *stop = buf + cut[t + 1];
		while (p < stop) {
			const char *eol = (const char *)memchr(p, '\n', stop - p);
			if (!eol) eol = stop;
			float y = 0.f;
			char at = 0;
			const size_t before = P.ents.size();
			const int rc = parse_line(p, eol, &y, P.ents, &P.maxf, &at);
			if (rc < 0) {
				P.err.pos = p - buf;
				P.err.msg = "cannot parse line \"" + std::string(p, eol) + "\" at character " + std::string(1, at);
				return;
			}
			if (rc > 0) {
				if (P.ents.size() > before) P.has_feature = true;
				P.mn = std::min(y, P.mn);   // Data.h:200-201
				P.mx = std::max(y, P.mx);
				if (y != y) P.has_nan = true;
				P.target.push_back(y);
				P.len.push_back((uint32_t)(P.ents.size() - before));
			}
			p = eol + 1;
		}
	});
	free(buf);
	for (const Part &P : part)
		if (P.err.pos != SIZE_MAX) { g_host_err = P.err.msg; return -1; }
	memset(out, 0, sizeof(*out));
	uint64_t nrows = 0, nnz = 0;
	int maxf = -1;
	bool has_feature = false;
	float mn = 3.40282347e+38f, mx = -3.40282347e+38f;
	std::vector<uint64_t> row0(T + 1, 0), ent0(T + 1, 0);
	for (int t = 0; t < T; t++) {
		row0[t + 1] = row0[t] + part[t].target.size();
		ent0[t + 1] = ent0[t] + part[t].ents.size();
		maxf = std::max(maxf, part[t].maxf);
		has_feature |= part[t].has_feature;
		// std::min(y, m) is not associative once a NaN appears (the fold returns the NaN, then
		// restarts from the next value), so a part holding a NaN target replaces the running
		// range: its own fold does not depend on where it started
		if (part[t].has_nan) { mn = part[t].mn; mx = part[t].mx; }
		else if (!part[t].target.empty()) { mn = std::min(part[t].mn, mn); mx = std::max(part[t].mx, mx); }
	}
	nrows = row0[T]; nnz = ent0[T];
	if (nrows > 0xFFFFFFFFull) { g_host_err = "too many rows"; return -1; }
	out->num_rows = (uint32_t)nrows;
	out->nnz = nnz;
	out->num_feature = has_feature ? (uint32_t)maxf + 1 : 0;   // Data.h:220-222
	out->min_target = mn;
	out->max_target = mx;
	out->target = xalloc<float>(nrows);
	out->row_ptr = xalloc<uint64_t>(nrows + 1);
	out->row_ent = xalloc<vbfm_entry>(nnz);
	out->row_ptr[0] = 0;
	parallel(T, [&](int t) {
		const Part &P = part[t];
		if (!P.target.empty()) memcpy(out->target + row0[t], P.target.data(), P.target.size() * sizeof(float));
		if (!P.ents.empty()) memcpy(out->row_ent + ent0[t], P.ents.data(), P.ents.size() * sizeof(vbfm_entry));
		uint64_t a = ent0[t];
		for (size_t i = 0; i < P.len.size(); i++) { a += P.len[i]; out->row_ptr[row0[t] + i + 1] = a; }
	});
	part.clear();
	transpose(out);
	return 0;
}

#pragma pack(push, 1)
struct sparse_header { uint32_t id, float_size; uint64_t num_values; uint32_t num_rows, num_cols; };
#pragma pack(pop)
static_assert(sizeof(sparse_header) == 24, "fmatrix.h file_header is 24 bytes");

// LargeSparseMatrixHD file (fmatrix.h:46-52, 66-82): header, then per row {uint32 size, entries}
int read_sparse(const std::string &fn, uint32_t *nrows, uint32_t *ncols, uint64_t *nnz, uint64_t **ptr,
                vbfm_entry **ent)
{
	FILE *fp = fopen(fn.c_str(), "rb");
	if (!fp) { g_host_err = "could not open " + fn; return -1; }
	sparse_header h;
	if (fread(&h, sizeof(h), 1, fp) != 1 || h.id != 2 || h.float_size != sizeof(float)) {
		fclose(fp);
		g_host_err = "bad sparse matrix header in " + fn;
		return -1;
	}
	*nrows = h.num_rows; *ncols = h.num_cols; *nnz = h.num_values;
	*ptr = xalloc<uint64_t>((size_t)h.num_rows + 1);
	*ent = xalloc<vbfm_entry>(h.num_values);
	(*ptr)[0] = 0;
	uint64_t c = 0;
	for (uint32_t r = 0; r < h.num_rows; r++) {
		uint32_t sz;
		if (fread(&sz, 4, 1, fp) != 1 || c + sz > h.num_values ||
		    fread(*ent + c, sizeof(vbfm_entry), sz, fp) != sz) {
			fclose(fp);
			g_host_err = "truncated sparse matrix " + fn;
			return -1;
		}
		c += sz;
		(*ptr)[r + 1] = c;
	}
	fclose(fp);
	if (c != h.num_values) { g_host_err = "value count mismatch in " + fn; return -1; }
	return 0;
}

int load_binary(const std::string &base, const char *ex, const char *ext, const char *ey, vbfm_host_data *out)
{
	memset(out, 0, sizeof(*out));
	// DVector::loadFromBinaryFile (matrix.h:296-312): uint32 version=1, size=4, n; floats
	FILE *fp = fopen((base + ey).c_str(), "rb");
	if (!fp) { g_host_err = "could not open " + base + ey; return -1; }
	uint32_t hdr[3];
	if (fread(hdr, 4, 3, fp) != 3 || hdr[0] != 1 || hdr[1] != sizeof(float)) {
		fclose(fp);
		g_host_err = "bad target file " + base + ey;
		return -1;
	}
	out->num_rows = hdr[2];
	out->target = xalloc<float>(hdr[2]);
	if (fread(out->target, 4, hdr[2], fp) != hdr[2]) { fclose(fp); g_host_err = "truncated " + base + ey; return -1; }
	fclose(fp);
	uint32_t xr, xc, tr, tc;
	uint64_t xn, tn;
	if (read_sparse(base + ex, &xr, &xc, &xn, &out->row_ptr, &out->row_ent)) return -1;
	if (read_sparse(base + ext, &tr, &tc, &tn, &out->col_ptr, &out->col_ent)) return -1;
	if (xr != out->num_rows || tc != xr || tr != xc || tn != xn) {   // Data.h:156-160
		g_host_err = "inconsistent binary data set " + base;
		return -1;
	}
	out->nnz = xn;
	out->num_feature = tr;   // Data.h:150: num_feature = data_t->getNumRows()
	out->min_target = 3.40282347e+38f;
	out->max_target = -3.40282347e+38f;
	for (uint32_t i = 0; i < out->num_rows; i++) {   // Data.h:161-166
		out->min_target = std::min(out->target[i], out->min_target);
		out->max_target = std::max(out->target[i], out->max_target);
	}
	return 0;
}

// LargeSparseMatrix::saveToBinaryFile (fmatrix.h:67-86): header, then per row {uint32 size, entries}
int write_sparse(const std::string &fn, uint32_t nrows, uint32_t ncols, uint64_t nnz, const uint64_t *ptr,
                 const vbfm_entry *ent)
{
	FILE *fp = fopen(fn.c_str(), "wb");
	if (!fp) { g_host_err = "could not open " + fn; return -1; }
	sparse_header h{2u, (uint32_t)sizeof(float), nnz, nrows, ncols};
	bool ok = fwrite(&h, sizeof(h), 1, fp) == 1;
	for (uint32_t r = 0; ok && r < nrows; r++) {
		const uint32_t sz = (uint32_t)(ptr[r + 1] - ptr[r]);
		ok = fwrite(&sz, 4, 1, fp) == 1 && (sz == 0 || fwrite(ent + ptr[r], sizeof(vbfm_entry), sz, fp) == sz);
	}
	ok = (fclose(fp) == 0) && ok;
	if (!ok) { g_host_err = "could not write " + fn; return -1; }
	return 0;
}

}  // namespace

extern "C" {

int vbfm_save_data(const char *basename, const vbfm_host_data *d)
{
	if (!basename || !d) { g_host_err = "vbfm_save_data: null argument"; return -1; }
	const std::string base(basename);
	// DVector::saveToBinaryFile (matrix.h:280-293): uint32 version 1, size 4, n; floats
	FILE *fp = fopen((base + ".y").c_str(), "wb");
	if (!fp) { g_host_err = "could not open " + base + ".y"; return -1; }
	const uint32_t hdr[3] = {1u, (uint32_t)sizeof(float), d->num_rows};
	bool ok = fwrite(hdr, 4, 3, fp) == 3 && (d->num_rows == 0 || fwrite(d->target, 4, d->num_rows, fp) == d->num_rows);
	ok = (fclose(fp) == 0) && ok;
	if (!ok) { g_host_err = "could not write " + base + ".y"; return -1; }
	if (write_sparse(base + ".x", d->num_rows, d->num_feature, d->nnz, d->row_ptr, d->row_ent)) return -1;
	return write_sparse(base + ".xt", d->num_feature, d->num_rows, d->nnz, d->col_ptr, d->col_ent);
}

const char *vbfm_host_last_error(void) { return g_host_err.c_str(); }
void vbfm_host_set_error(const char *msg) { g_host_err = msg ? msg : ""; }

int vbfm_load_data(const char *filename, vbfm_host_data *out)
{
	const std::string base(filename);
	// Data.h:112-117: .data/.datat/.target first, then .x/.xt/.y, else text
	if (file_exists(base + ".data") && file_exists(base + ".datat") && file_exists(base + ".target"))
		return load_binary(base, ".data", ".datat", ".target", out);
	if (file_exists(base + ".x") && file_exists(base + ".xt") && file_exists(base + ".y"))
		return load_binary(base, ".x", ".xt", ".y", out);
	return load_text(filename, out);
}

void vbfm_free_host_data(vbfm_host_data *d)
{
	if (!d) return;
	free(d->target); free(d->row_ptr); free(d->row_ent); free(d->col_ptr); free(d->col_ent);
	memset(d, 0, sizeof(*d));
}

int vbfm_init_params_host(uint32_t seed, double init_stdev, int32_t k, uint32_t D, uint32_t G, vbfm_params *p,
                          double *fm_v, double *fm_w)
{
	if (!p || !p->mu_w || !p->sigma_w || (k > 0 && (!p->mu_v || !p->sigma_v)) || !p->hyp_sigma_w ||
	    (k > 0 && !p->hyp_sigma_v)) {
		g_host_err = "vbfm_init_params_host: output arrays missing";
		return -1;
	}
	const size_t kd = (size_t)k * D;
	vbrng::Glibc rng(seed);                                            // srand(seed), libfm.cpp:123-124
	for (size_t i = 0; i < kd; i++) {                                  // fm_model::init (fm_model.h:97)
		const double v = rng.gaussian(0, init_stdev);
		if (fm_v) fm_v[i] = v;
	}
	for (uint32_t i = 0; i < D; i++) {                                 // libfm.cpp:307
		const double w = rng.gaussian(0, init_stdev);
		if (fm_w) fm_w[i] = w;
	}
	// fm_learn_vb::init (fm_learn_vb.h:693-712)
	p->alpha = 1.0; p->sigma_0 = 1.0; p->mu_0_dash = 0.0; p->sigma_0_dash = 0.02;
	for (uint32_t g = 0; g < G; g++) p->hyp_sigma_w[g] = 1;
	for (size_t i = 0; i < (size_t)G * k; i++) p->hyp_sigma_v[i] = 1;
	for (uint32_t i = 0; i < D; i++) p->mu_w[i] = 0.1 * rng.gaussian(0, 1);   // DVectorDoubleVB::init_normal
	for (uint32_t i = 0; i < D; i++) p->sigma_w[i] = .02;
	for (size_t i = 0; i < kd; i++) p->mu_v[i] = 0.1 * rng.gaussian(0, 1);   // DMatrixDoubleVB::init_normal
	for (size_t i = 0; i < kd; i++) p->sigma_v[i] = .02;
	return 0;
}

}  // extern "C"
