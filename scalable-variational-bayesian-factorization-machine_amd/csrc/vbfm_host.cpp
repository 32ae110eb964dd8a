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
#include <string>
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

// one text line: "<target> <id>:<value> ..." (Data.h:196-215 / 247-272)
int parse_line(const char *line, float *target, std::vector<vbfm_entry> &ents, int *maxf)
{
	const char *p = line;
	while (*p == ' ' || *p == '\t') p++;
	if (*p == 0 || *p == '#') return 0;
	float v;
	int nchar, fid;
	if (sscanf(p, "%f%n", &v, &nchar) < 1) return -1;
	p += nchar;
	*target = v;
	while (sscanf(p, "%d:%f%n", &fid, &v, &nchar) >= 2) {
		p += nchar;
		if (fid < 0) return -2;
		if (fid > *maxf) *maxf = fid;
		ents.push_back(vbfm_entry{(uint32_t)fid, v});
	}
	while (*p != 0 && (*p == ' ' || *p == '\t')) p++;
	if (*p != 0 && *p != '#') return -1;
	return 1;
}

template <class T> T *xalloc(size_t n) { return (T *)malloc((n ? n : 1) * sizeof(T)); }

// Data::create_data_t (Data.h:457-509): stable counting transpose, ascending rows per column
void transpose(vbfm_host_data *d)
{
	const uint32_t nf = d->num_feature;
	d->col_ptr = xalloc<uint64_t>((size_t)nf + 1);
	d->col_ent = xalloc<vbfm_entry>(d->nnz);
	std::vector<uint64_t> cnt((size_t)nf + 1, 0);
	for (uint64_t j = 0; j < d->nnz; j++) cnt[d->row_ent[j].id]++;
	d->col_ptr[0] = 0;
	for (uint32_t i = 0; i < nf; i++) d->col_ptr[i + 1] = d->col_ptr[i] + cnt[i];
	for (uint32_t i = 0; i < nf; i++) cnt[i] = d->col_ptr[i];
	for (uint32_t r = 0; r < d->num_rows; r++)
		for (uint64_t j = d->row_ptr[r]; j < d->row_ptr[r + 1]; j++) {
			const vbfm_entry &e = d->row_ent[j];
			d->col_ent[cnt[e.id]++] = vbfm_entry{r, e.value};
		}
}

int load_text(const char *fn, vbfm_host_data *out)
{
	FILE *fp = fopen(fn, "r");
	if (!fp) { g_host_err = std::string("unable to open ") + fn; return -1; }
	std::vector<vbfm_entry> ents;
	std::vector<float> target;
	std::vector<uint64_t> row_ptr(1, 0);
	int maxf = -1;
	bool has_feature = false;
	float mn = 3.40282347e+38f, mx = -3.40282347e+38f;
	char *line = nullptr;
	size_t cap = 0;
	ssize_t len;
	while ((len = getline(&line, &cap, fp)) >= 0) {
		if (len > 0 && line[len - 1] == '\n') line[len - 1] = 0;
		float y;
		const size_t before = ents.size();
		const int rc = parse_line(line, &y, ents, &maxf);
		if (rc < 0) {
			g_host_err = std::string("cannot parse line \"") + line + "\"";
			free(line); fclose(fp);
			return -1;
		}
		if (rc == 0) continue;
		if (ents.size() > before) has_feature = true;
		mn = std::min(y, mn);
		mx = std::max(y, mx);
		target.push_back(y);
		row_ptr.push_back(ents.size());
	}
	free(line);
	fclose(fp);
	memset(out, 0, sizeof(*out));
	out->num_rows = (uint32_t)target.size();
	out->nnz = ents.size();
	out->num_feature = has_feature ? (uint32_t)maxf + 1 : 0;   // Data.h:220-222
	out->min_target = mn;
	out->max_target = mx;
	out->target = xalloc<float>(target.size());
	memcpy(out->target, target.data(), target.size() * sizeof(float));
	out->row_ptr = xalloc<uint64_t>(row_ptr.size());
	memcpy(out->row_ptr, row_ptr.data(), row_ptr.size() * sizeof(uint64_t));
	out->row_ent = xalloc<vbfm_entry>(ents.size());
	memcpy(out->row_ent, ents.data(), ents.size() * sizeof(vbfm_entry));
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

}  // namespace

extern "C" {

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
