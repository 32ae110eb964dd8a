// host/libfm_main.cpp -- drop-in for the reference's `bin/libFM -method vb | vb_online | mcmc | als`
// on MI355X.
//
// Mirrors main() of src/libfm/libfm.cpp (flag surface, defaults, RNG order, output lines and
// files) and the iteration loop of fm_learn_vb_simultaneous::_learn
// (src/libfm/src/fm_learn_vb_simultaneous.h:18-259); the learner itself is libvbfm.so
// (include/vbfm.h). Deliberate differences, all documented in INTEGRATION.md:
//   * -seed is honoured (the reference seeds with time(NULL) and ignores it, libfm.cpp:123);
//   * -out writes the clipped test predictions of the last iteration (the reference's VB
//     predict() body is commented out and leaves the vector uninitialised, fm_learn_vb.h:321);
//   * -method sgd/sgda/... and -task c are rejected with an error instead of running
//     other learners; -relation is not supported;
//   * extra flags: -device (HIP ordinal), -vfile 0 (skip writing v_file.txt), -save_state /
//     -resume (checkpoints), -parity_log (17-digit JSON lines per iteration), and the multi-GPU launch: -devices N | o0,o1,..., -shard
//     rows|features, -transport rccl|host, -plan 1 (print the ranks' shard plan, no GPU).
//
// Multi-GPU (-devices): the reference is one process on one core. Here this process parses the
// flags and loads the data (host code only, no HIP call), then forks one rank process per GPU
// BEFORE anything touches a GPU; each rank hands its slice of the train and test rows to its
// own libvbfm context (row shards: rows [N r/P, N (r+1)/P), the exact mode) or all rows
// (feature shards) and joins the communicator: RCCL over xGMI (rank 0's ncclUniqueId travels
// through a shared-memory page) or, with -transport host, an all-reduce through shared memory
// (several ranks may then share one GPU, which RCCL refuses). Rank 0 prints the reference's
// lines and writes its files; this process waits, and kills the other ranks when one fails.
#include "../../include/vbfm.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <algorithm>
#include <csignal>
#include <cstring>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/wait.h>
#include <unistd.h>
#include <vector>

namespace {

// CMDLine (src/util/cmdline.h:29-197): "-name value", "--name", lists split on ";,".
class CmdLine {
public:
	std::map<std::string, std::string> help, value;
	CmdLine(int argc, char **argv)
	{
		int i = 1;
		while (i < argc) {
			std::string s(argv[i]);
			if (!parse_name(s)) throw std::string("cannot parse " + s);
			if (value.count(s)) throw std::string("the parameter " + s + " is already specified");
			if (i + 1 < argc) {
				std::string nx(argv[i + 1]);
				if (!parse_name(nx)) { value[s] = argv[i + 1]; i++; }
				else value[s] = "";
			} else value[s] = "";
			i++;
		}
	}
	static bool parse_name(std::string &s)
	{
		if (s.size() > 0 && s[0] == '-') {
			s = (s.size() > 1 && s[1] == '-') ? s.substr(2) : s.substr(1);
			return true;
		}
		return false;
	}
	const std::string &reg(const std::string &p, const std::string &h) { help[p] = h; return p; }
	bool has(const std::string &p) const { return value.count(p) > 0; }
	void check() const
	{
		for (const auto &kv : value)
			if (!help.count(kv.first)) throw std::string("the parameter " + kv.first + " does not exist");
	}
	std::string get(const std::string &p, const std::string &d = "") const { return has(p) ? value.at(p) : d; }
	double getd(const std::string &p, double d) const { return has(p) ? atof(value.at(p).c_str()) : d; }
	long geti(const std::string &p, long d) const { return has(p) ? atoi(value.at(p).c_str()) : d; }
	std::vector<std::string> list(const std::string &p) const
	{
		std::vector<std::string> out;
		const std::string s = get(p);
		size_t a = s.find_first_not_of(";,");
		while (a != std::string::npos) {
			size_t b = s.find_first_of(";,", a);
			out.push_back(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
			a = s.find_first_not_of(";,", b);
		}
		return out;
	}
	void print_help() const
	{
		for (const auto &kv : help) {
			std::cout << "-" << kv.first;
			for (size_t i = kv.first.size() + 1; i < 16; i++) std::cout << " ";
			std::cout << kv.second << std::endl;
		}
	}
};

// RLog (src/util/rlog.h:29-91): TSV of registered fields, one line per iteration
class RLog {
public:
	explicit RLog(std::ostream *o) : out(o) {}
	void add(const std::string &f) { header.push_back(f); value[f] = NAN; }
	void log(const std::string &f, double d) { value[f] = d; }
	void init()
	{
		for (size_t i = 0; i < header.size(); i++) *out << header[i] << (i + 1 < header.size() ? "\t" : "\n");
		out->flush();
	}
	void newline()
	{
		for (size_t i = 0; i < header.size(); i++) *out << value[header[i]] << (i + 1 < header.size() ? "\t" : "\n");
		out->flush();
		for (auto &kv : value) kv.second = NAN;
	}
private:
	std::ostream *out;
	std::vector<std::string> header;
	std::map<std::string, double> value;
};

// -parity_log FILE ("Metrics / logging"): a first line {"method": "setup", ...} with the
// set-up costs (plog_setup, every method), then one JSON line per iteration from rank 0 with
// the values the reference prints, at 17 significant digits (its test_rmse_* / free_energy_*
// files carry 6, too few for a 1e-6 comparison), the device time of the phases, and the factor
// sweep's throughput: nnz*k per second of ms_v over the whole job and, per GPU, the fraction of
// the 8 TB/s HBM roofline by SURVEY §8d's bytes model (VB B = 128 nnz + 24 N + 32 D per factor,
// MCMC / ALS 72 nnz + 8 N + 16 D). Non-finite values are written as null.
class ParityLog {
public:
	ParityLog(const std::string &path, bool lead)
	{
		if (path.empty() || !lead) return;
		f = fopen(path.c_str(), "w");
		if (!f) throw std::string("Unable to open file " + path);
	}
	~ParityLog() { if (f) fclose(f); }
	ParityLog(const ParityLog &) = delete;
	ParityLog &operator=(const ParityLog &) = delete;
	bool on() const { return f != nullptr; }
	void begin(const char *method, uint32_t it)
	{
		line = std::string("\"method\": \"") + method + "\"";
		num("iter", (double)it);
	}
	void str(const char *key, const char *v) { line += std::string(", \"") + key + "\": \"" + v + "\""; }
	void num(const char *key, double v)
	{
		char b[48];
		if (std::isfinite(v)) snprintf(b, sizeof(b), "%.17g", v);
		else snprintf(b, sizeof(b), "null");
		line += std::string(", \"") + key + "\": " + b;
	}
	// the factor sweep of one iteration: ms_v of rank 0, the whole job's nnz, rows and features
	void sweep(double ms_v, int k, uint64_t nnz, uint32_t rows, uint32_t nf, int ranks, bool mcmc)
	{
		const double s = ms_v * 1e-3;
		const double bytes = mcmc ? 72.0 * nnz + 8.0 * rows + 16.0 * nf : 128.0 * nnz + 24.0 * rows + 32.0 * nf;
		num("sweep_nnz_k_per_s", s > 0 ? (double)nnz * k / s : NAN);
		num("hbm_frac_per_gpu", s > 0 ? bytes * k / ranks / s / 8e12 : NAN);
	}
	// the iteration's exchanges over the ranks (vbfm_exchange_info): all-reduces, their payload per
	// rank and their time (RCCL: the sampled ones scaled to all; host exchange: every call)
	void exchange(vbfm_ctx *ctx);
	void end()
	{
		fprintf(f, "{%s}\n", line.c_str());
		fflush(f);
	}
private:
	FILE *f = nullptr;
	std::string line;
};

// host wall seconds of the train and test loads (Data::load, libfm.cpp:149-171), for -parity_log
static double g_load_s = 0;

static double wall_now()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (double)ts.tv_sec + ts.tv_nsec * 1e-9;
}

void check(int rc, vbfm_ctx *ctx);

void ParityLog::exchange(vbfm_ctx *ctx)
{
	vbfm_exchange_stats xs;
	check(vbfm_exchange_info(ctx, &xs), ctx);
	num("exchange_calls", (double)xs.n_calls);
	num("exchange_bytes", (double)xs.bytes);
	num("ms_exchange", xs.ms_estimated);
	num("exchange_timed", xs.n_timed);
}

// -parity_log's first line: what setting the train set up cost (vbfm_setup_info): the load, the
// hand-over to the device, the dependency levels, the row store and its placement search
static void plog_setup(ParityLog &plog, vbfm_ctx *ctx, const char *method)
{
	if (!plog.on()) return;
	vbfm_setup_stats su;
	check(vbfm_setup_info(ctx, &su), ctx);
	plog.begin("setup", 0);
	plog.str("learner", method);
	plog.num("load_s", g_load_s);
	plog.num("set_train_s", su.s_set_train);
	plog.num("schedule_s", su.s_schedule);
	plog.num("store_s", su.s_store);
	plog.num("placement_s", su.s_placement);
	plog.num("placement_bytes", (double)su.place_bytes);
	plog.num("placement_candidates", su.place_candidates);
	plog.num("placement_kept_0", su.place_kept[0]);
	plog.num("placement_kept_1", su.place_kept[1]);
	plog.end();
}

double usertime()
{
	struct rusage ru;
	getrusage(RUSAGE_SELF, &ru);
	return (double)ru.ru_utime.tv_sec + (double)ru.ru_utime.tv_usec / 1000000.0;
}

struct Data {
	vbfm_host_data h{};
	~Data() { vbfm_free_host_data(&h); }
	vbfm_csc csc() const { return vbfm_csc{h.num_rows, h.num_feature, h.nnz, h.col_ptr, h.col_ent, h.target}; }
};

void check(int rc, vbfm_ctx *ctx)
{
	if (rc != 0) throw std::string(vbfm_last_error(ctx));
}

void load(const std::string &fn, Data &d, const char *what)
{
	std::cout << "Loading " << what << "...\t" << std::endl;
	if (vbfm_load_data(fn.c_str(), &d.h) != 0) throw std::string(vbfm_last_error(nullptr));
	std::cout << "num_rows=" << d.h.num_rows << "\tnum_values=" << d.h.nnz << "\tnum_features=" << d.h.num_feature
	          << "\tmin_target=" << d.h.min_target << "\tmax_target=" << d.h.max_target << std::endl;
}

// ---- ranks ------------------------------------------------------------------------------
// The shared-memory page the forked ranks use: a process-shared barrier, rank 0's RCCL
// unique id, one slot per rank for the host all-reduce, and the gathered test predictions
// (-out). Created by the launching process before fork (MAP_SHARED | MAP_ANONYMOUS).
struct ShmHeader {
	pthread_barrier_t bar;
	uint8_t uid[128];
	uint64_t slot_bytes;
	int32_t nranks;
};

struct Slice {   // one rank's rows of a data set as the C-ABI takes them
	std::vector<uint64_t> cp;
	std::vector<vbfm_entry> ent;
	std::vector<float> y;
	vbfm_csc csc{};
};

struct Rank {
	int32_t rank = 0, nranks = 1;
	int32_t device = 0;            // HIP ordinal of this rank (-1: rank % visible devices, resolved in the rank)
	bool host = false;             // -transport host
	int32_t shard = VBFM_SHARD_ROWS;
	ShmHeader *shm = nullptr;
	char *slots = nullptr;         // nranks x slot_bytes
	double *test_pred = nullptr;   // [test rows] gathered predictions
	bool lead() const { return rank == 0; }
	bool multi() const { return nranks > 1; }
	bool row_shards() const { return multi() && shard == VBFM_SHARD_ROWS; }
	void barrier() const
	{
		if (shm) pthread_barrier_wait(&shm->bar);
	}
	// this rank's rows [lo, hi) of n (row shards; all rows otherwise)
	void range(uint32_t n, uint32_t *lo, uint32_t *hi) const
	{
		if (!row_shards()) { *lo = 0; *hi = n; return; }
		*lo = (uint32_t)((uint64_t)n * rank / nranks);
		*hi = (uint32_t)((uint64_t)n * (rank + 1) / nranks);
	}
	// the rank's slice of a loaded data set: each column's entries of rows [lo, hi) (a
	// contiguous run: create_data_t lists a column's rows in ascending order, Data.h:457-509),
	// row ids made local, every column kept (the feature count stays global)
	Slice slice(const vbfm_host_data &h) const
	{
		Slice s;
		uint32_t lo, hi;
		range(h.num_rows, &lo, &hi);
		if (lo == 0 && hi == h.num_rows) {   // every row: the loaded arrays themselves (no copy of nnz entries)
			s.csc = vbfm_csc{h.num_rows, h.num_feature, h.nnz, h.col_ptr, h.col_ent, h.target};
			return s;
		}
		s.cp.assign((size_t)h.num_feature + 1, 0);
		auto run = [&](uint32_t j, const vbfm_entry **a, const vbfm_entry **z) {
			const vbfm_entry *b = h.col_ent + h.col_ptr[j], *e = h.col_ent + h.col_ptr[j + 1];
			*a = std::lower_bound(b, e, lo, [](const vbfm_entry &x, uint32_t r) { return x.id < r; });
			*z = std::lower_bound(*a, e, hi, [](const vbfm_entry &x, uint32_t r) { return x.id < r; });
		};
		for (uint32_t j = 0; j < h.num_feature; j++) {   // the slice's column pointers, then its entries
			const vbfm_entry *a, *z;
			run(j, &a, &z);
			s.cp[j + 1] = s.cp[j] + (uint64_t)(z - a);
		}
		s.ent.resize(s.cp[h.num_feature]);
		for (uint32_t j = 0; j < h.num_feature; j++) {
			const vbfm_entry *a, *z;
			run(j, &a, &z);
			vbfm_entry *o = s.ent.data() + s.cp[j];
			for (const vbfm_entry *p = a; p < z; p++) *o++ = vbfm_entry{p->id - lo, p->value};
		}
		s.y.assign(h.target + lo, h.target + hi);
		s.csc = vbfm_csc{hi - lo, h.num_feature, (uint64_t)s.ent.size(), s.cp.data(), s.ent.data(), s.y.data()};
		return s;
	}
	// a per-rank file name for -save_state / -resume (one checkpoint per rank)
	std::string rank_file(const std::string &path) const
	{
		return multi() ? path + "." + std::to_string(rank) : path;
	}
};

// host all-reduce through the shared slots: every rank copies its chunk into its slot, then
// every rank reduces the slots in rank order 0..P-1 (the same arithmetic on every rank, so
// all ranks hold identical results), chunk by chunk
template <typename T>
void reduce_slots(const Rank &rk, T *out, size_t n, size_t stride, int32_t op)
{
	for (size_t i = 0; i < n; i++) {
		T acc = ((const T *)rk.slots)[i];
		for (int32_t r = 1; r < rk.nranks; r++) {
			const T v = ((const T *)(rk.slots + (size_t)r * stride))[i];
			acc = op == VBFM_X_MAX ? std::max(acc, v) : (T)(acc + v);
		}
		out[i] = acc;
	}
}

int shm_exchange(void *user, void *buf, uint64_t count, int32_t dtype, int32_t op)
{
	const Rank &rk = *(const Rank *)user;
	const size_t es = dtype == VBFM_X_F64 ? 8 : dtype == VBFM_X_U32 ? 4 : 1;
	const size_t stride = rk.shm->slot_bytes, per = stride / es;
	char *b = (char *)buf;
	for (uint64_t off = 0; off < count; off += per) {
		const size_t n = (size_t)std::min<uint64_t>(per, count - off);
		memcpy(rk.slots + (size_t)rk.rank * stride, b + off * es, n * es);
		rk.barrier();
		if (dtype == VBFM_X_F64) reduce_slots(rk, (double *)(b + off * es), n, stride, op);
		else if (dtype == VBFM_X_U32) reduce_slots(rk, (uint32_t *)(b + off * es), n, stride, op);
		else reduce_slots(rk, (uint8_t *)(b + off * es), n, stride, op);
		rk.barrier();   // no slot is overwritten before every rank has read it
	}
	return 0;
}

// the rank joins its communicator (before vbfm_set_train) and picks the shard mode
void join(vbfm_ctx *ctx, const Rank &rk)
{
	if (!rk.multi()) return;
	check(vbfm_set_shard_mode(ctx, rk.shard, 0), ctx);
	if (rk.host) {
		check(vbfm_comm_init_host(ctx, rk.nranks, rk.rank, shm_exchange, (void *)&rk), ctx);
		return;
	}
	if (rk.lead()) check(vbfm_comm_unique_id(rk.shm->uid), nullptr);
	rk.barrier();
	check(vbfm_comm_init(ctx, rk.nranks, rk.rank, rk.shm->uid), ctx);
}

// test predictions of every rank into the shared array (row shards): rank 0 then has them all
void gather_test(const Rank &rk, const Data &test, const std::vector<double> &local, std::vector<double> *all)
{
	if (!rk.row_shards()) { *all = local; return; }
	uint32_t lo, hi;
	rk.range(test.h.num_rows, &lo, &hi);
	std::copy(local.begin(), local.end(), rk.test_pred + lo);
	rk.barrier();
	if (rk.lead()) all->assign(rk.test_pred, rk.test_pred + test.h.num_rows);
	rk.barrier();
}

}  // namespace

// -method mcmc | als (libfm.cpp:131-135, 297-305, 367-411; fm_learn_mcmc_simultaneous.h:50-305)
struct McmcRun {
	bool sample;
	uint32_t seed;
	double init_stdev;
	uint32_t num_iter;
	std::vector<double> reg;
	const uint32_t *groups;
	uint32_t G, D;
	int k0, k1, k;
	bool vfile;
	std::string rlog_file, out_file, parity_file, save_file, resume_file;
};

static void run_mcmc(const McmcRun &r, Data &train, Data &test, const Rank &rk)
{
	vbfm_ctx *ctx = nullptr;
	try {
		vbfm_config cfg{r.k0, r.k1, r.k, r.D, r.G, r.groups, train.h.min_target, train.h.max_target, rk.device, 0};
		check(vbfm_create(&ctx, &cfg), nullptr);
		join(ctx, rk);
		{
			const Slice tr = rk.slice(train.h), te = rk.slice(test.h);
			check(vbfm_set_train(ctx, &tr.csc), ctx);
			check(vbfm_set_test(ctx, &te.csc), ctx);
		}
		vbfm_mcmc_config mc{r.sample, r.sample, VBFM_RNG_REFERENCE, r.seed, r.init_stdev,
		                    r.reg.empty() ? nullptr : r.reg.data(), (int32_t)r.reg.size()};
		check(vbfm_mcmc_init(ctx, &mc), ctx);
		const size_t kd = (size_t)r.k * r.D, gk = (size_t)r.G * r.k;
		std::vector<double> w(r.D), v(kd), wmu(r.G), wl(r.G), vmu(gk), vl(gk);
		vbfm_mcmc_params p{w.data(), v.data(), wmu.data(), wl.data(), vmu.data(), vl.data(), 0, 0, 0};
		const bool resume = !r.resume_file.empty();
		if (r.vfile && rk.lead() && !resume) {   // fm_model.h:98: the initial factors (DMatrix::save, matrix.h:129-152)
			check(vbfm_mcmc_get_params(ctx, &p), ctx);
			std::ofstream vf("v_file.txt");
			for (int f = 0; f < r.k; f++) {
				for (uint32_t j = 0; j < r.D; j++) vf << (j ? "\t" : "") << v[(size_t)f * r.D + j];
				vf << std::endl;
			}
		}
		std::ofstream *rlog_out = nullptr;
		RLog *rlog = nullptr;
		if (!r.rlog_file.empty() && rk.lead()) {   // fm_learn::init + fm_learn_mcmc::init fields (:1118-1149)
			rlog_out = new std::ofstream(r.rlog_file.c_str());
			if (!rlog_out->is_open()) throw std::string("Unable to open file " + r.rlog_file);
			std::cout << "logging to " << r.rlog_file << std::endl;
			rlog = new RLog(rlog_out);
			for (const char *f : {"rmse", "mae", "time_pred", "time_learn", "time_learn2", "time_learn4", "alpha",
			                      "rmse_mcmc_this", "rmse_mcmc_all", "rmse_mcmc_all_but5"})
				rlog->add(f);
			for (uint32_t g = 0; g < r.G; g++) {
				std::ostringstream ss;
				ss << "wmu[" << g << "]"; rlog->add(ss.str()); ss.str("");
				ss << "wlambda[" << g << "]"; rlog->add(ss.str()); ss.str("");
				for (int f = 0; f < r.k; f++) {
					ss << "vmu[" << g << "," << f << "]"; rlog->add(ss.str()); ss.str("");
					ss << "vlambda[" << g << "," << f << "]"; rlog->add(ss.str()); ss.str("");
				}
			}
			rlog->init();
		}
		std::cout << "in mcmc learn" << std::endl << "preprocess complete" << std::endl;
		// -resume: the chain's state from the file instead of the initial caches (the initial
		// draws above are replaced by the file's parameters and RNG position)
		uint32_t it0 = 0;
		if (resume) {
			check(vbfm_load_state(ctx, rk.rank_file(r.resume_file).c_str(), &it0), ctx);
			std::cout << "resuming from " << r.resume_file << " after " << it0 << " iterations" << std::endl;
		} else {
			check(vbfm_mcmc_init_caches(ctx), ctx);
		}
		std::ostringstream tag;
		tag << r.k0 << r.k1 << r.k;
		const std::string f_rmse = "test_rmse_" + tag.str() + "_mcmc";
		if (rk.lead() && !resume) { std::ofstream a(f_rmse.c_str()); }   // truncate (:52-62); a resumed run appends
		ParityLog plog(r.parity_file, rk.lead());
		plog_setup(plog, ctx, r.sample ? "mcmc" : "als");
		for (uint32_t it = it0; it < it0 + r.num_iter; it++) {
			const double t_user = usertime();
			const clock_t t_clock = clock();
			const double t_wall = (double)time(NULL);
			vbfm_mcmc_stats st;
			check(vbfm_mcmc_iterate(ctx, &st), ctx);
			// :104-127
			const struct { const char *name; uint32_t nan, inf; } rep[] = {
				{"alpha", st.nan_alpha, st.inf_alpha}, {"w0", st.nan_w0, st.inf_w0}, {"w", st.nan_w, st.inf_w},
				{"v", st.nan_v, st.inf_v}, {"w_mu", st.nan_w_mu, st.inf_w_mu},
				{"w_lambda", st.nan_w_lambda, st.inf_w_lambda}, {"v_mu", st.nan_v_mu, st.inf_v_mu},
				{"v_lambda", st.nan_v_lambda, st.inf_v_lambda}};
			for (const auto &q : rep)
				if (q.nan > 0 || q.inf > 0)
					std::cout << "#nans in " << q.name << ":\t" << q.nan << "\t#inf_in_" << q.name << ":\t" << q.inf
					          << std::endl;
			if (rlog) {
				check(vbfm_mcmc_get_params(ctx, &p), ctx);
				rlog->log("alpha", st.alpha);
				for (uint32_t g = 0; g < r.G; g++) {
					std::ostringstream ss;
					ss << "wmu[" << g << "]"; rlog->log(ss.str(), wmu[g]); ss.str("");
					ss << "wlambda[" << g << "]"; rlog->log(ss.str(), wl[g]); ss.str("");
					for (int f = 0; f < r.k; f++) {
						ss << "vmu[" << g << "," << f << "]"; rlog->log(ss.str(), vmu[(size_t)g * r.k + f]); ss.str("");
						ss << "vlambda[" << g << "," << f << "]"; rlog->log(ss.str(), vl[(size_t)g * r.k + f]); ss.str("");
					}
				}
				rlog->log("time_learn", usertime() - t_user);
				rlog->log("time_learn2", (double)(clock() - t_clock) / CLOCKS_PER_SEC);
				rlog->log("time_learn4", (double)time(NULL) - t_wall);
				rlog->log("rmse", st.rmse_all);
				rlog->log("mae", st.mae_all);
				rlog->log("rmse_mcmc_this", st.rmse_this);
				rlog->log("rmse_mcmc_all", st.rmse_all);
				rlog->newline();
			}
			std::cout << "#Iter=" << std::setw(3) << it << "\tTrain=" << st.train_rmse << "\tTest=" << st.rmse_all
			          << std::endl;
			if (plog.on()) {
				plog.begin(r.sample ? "mcmc" : "als", it);
				const double vals[] = {st.train_rmse, st.rmse_all, st.mae_all, st.rmse_this, st.mae_this, st.alpha, st.w0,
				                       st.ms_hyper, st.ms_w, st.ms_v, st.ms_predict, st.ms_total};
				const char *keys[] = {"train", "test_rmse", "test_mae", "test_rmse_this", "test_mae_this", "alpha", "w0",
				                      "ms_hyper", "ms_w", "ms_v", "ms_predict", "ms_total"};
				for (size_t i = 0; i < sizeof(vals) / sizeof(vals[0]); i++) plog.num(keys[i], vals[i]);
				plog.num("levels", st.num_levels);
				plog.num("rng_skipped", st.rng_skipped);
				plog.sweep(st.ms_v, r.k, train.h.nnz, train.h.num_rows, train.h.num_feature, rk.nranks, true);
				plog.exchange(ctx);
				plog.end();
			}
			if (rk.lead()) {
				std::ofstream fr(f_rmse.c_str(), std::ios_base::app);
				fr << st.rmse_all << "\n";
			}
		}
		if (!r.save_file.empty())
			check(vbfm_save_state(ctx, rk.rank_file(r.save_file).c_str(), it0 + r.num_iter), ctx);
		std::cout << "after learn" << std::endl;   // libfm.cpp:507; no Final line for mcmc (:509)
		if (!r.out_file.empty()) {                 // libfm.cpp:514-519
			uint32_t lo, hi;
			rk.range(test.h.num_rows, &lo, &hi);
			std::vector<double> pred(hi - lo), all;
			check(vbfm_mcmc_get_test_pred(ctx, (int32_t)(it0 + r.num_iter), pred.data()), ctx);
			gather_test(rk, test, pred, &all);
			if (rk.lead()) {
				std::ofstream o(r.out_file.c_str());
				for (double x : all) o << x << std::endl;
			}
		}
		delete rlog;
		delete rlog_out;
		vbfm_destroy(ctx);
	} catch (...) {
		if (ctx) vbfm_destroy(ctx);
		throw;
	}
}

// the reference's NaN reports (fm_learn_vb_simultaneous.h:89-118 and
// fm_learn_vb_online_simultaneous.h:159-188; labels as printed there)
static void nan_reports(uint32_t nan_alpha, uint32_t inf_alpha, uint32_t nan_mu_w, uint32_t inf_mu_w,
                        uint32_t nan_sigma_w, uint32_t nan_mu_v, uint32_t inf_mu_v, uint32_t nan_sigma_v)
{
	if (nan_alpha > 0 || inf_alpha > 0)
		std::cout << "#nans in alpha:\t" << nan_alpha << "\t#inf_in_alpha:\t" << inf_alpha << std::endl;
	if (nan_mu_w > 0 || inf_mu_w > 0)
		std::cout << "#nans in alpha:\t" << nan_mu_w << "\t#inf_in_alpha:\t" << inf_mu_w << std::endl;
	if (nan_sigma_w > 0) std::cout << "#nans in alpha:\t" << nan_sigma_w << "\t#inf_in_alpha:\t" << 0 << std::endl;
	if (nan_mu_v > 0 || inf_mu_v > 0)
		std::cout << "#nans in alpha:\t" << nan_mu_v << "\t#inf_in_alpha:\t" << inf_mu_v << std::endl;
	if (nan_sigma_v > 0) std::cout << "#nans in alpha:\t" << nan_sigma_v << "\t#inf_in_alpha:\t" << 0 << std::endl;
}

static void write_vfile(const std::vector<double> &fm_v, int k, uint32_t D)
{
	// fm_model.h:98 (DMatrix::save, matrix.h:129-152)
	std::ofstream vf("v_file.txt");
	for (int f = 0; f < k; f++) {
		for (uint32_t j = 0; j < D; j++) vf << (j ? "\t" : "") << fm_v[(size_t)f * D + j];
		vf << std::endl;
	}
}

// -method vb_online (libfm.cpp:159-171, 312-320, 494-503; fm_learn_vb_online_simultaneous.h:20-290)
struct OnlineRun {
	uint32_t seed;
	double init_stdev;
	uint32_t num_iter, num_batch;
	const uint32_t *groups;
	uint32_t G, D;
	int k0, k1, k;
	bool vfile;
	std::string rlog_file, out_file, parity_file, save_file, resume_file;
};

static void run_online(const OnlineRun &r, Data &train, Data &test, const Rank &rk)
{
	if (rk.multi()) throw std::string("-method vb_online runs on one GPU (-devices 1)");
	vbfm_ctx *ctx = nullptr;
	try {
		vbfm_config cfg{r.k0, r.k1, r.k, r.D, r.G, r.groups, train.h.min_target, train.h.max_target, rk.device, 0};
		check(vbfm_create(&ctx, &cfg), nullptr);
		const vbfm_csc tr = train.csc(), te = test.csc();
		check(vbfm_set_train(ctx, &tr), ctx);
		check(vbfm_set_test(ctx, &te), ctx);
		const size_t kd = (size_t)r.k * r.D;
		std::vector<double> fm_v(r.vfile ? kd : 0);
		const char *init_env = getenv("VBFM_INIT");
		const bool replay = init_env ? std::string(init_env) == "replay" : kd + r.D >= 2000000;
		vbfm_online_config oc{r.num_batch, r.seed, r.init_stdev,
		                      replay ? VBFM_ONLINE_INIT_REPLAY : VBFM_ONLINE_INIT_HOST, r.vfile ? fm_v.data() : nullptr};
		check(vbfm_online_init(ctx, &oc), ctx);
		const bool resume = !r.resume_file.empty();
		if (r.vfile && !resume) write_vfile(fm_v, r.k, r.D);
		// -resume: the learner's state (parameters, natural parameters, step sizes, the rand()
		// stream and the last permutation) from the file instead of the initial draws
		uint32_t it0 = 0;
		if (resume) {
			check(vbfm_load_state(ctx, r.resume_file.c_str(), &it0), ctx);
			std::cout << "resuming from " << r.resume_file << " after " << it0 << " iterations" << std::endl;
		}
		std::ofstream *rlog_out = nullptr;
		RLog *rlog = nullptr;
		if (!r.rlog_file.empty()) {   // fm_learn::init + fm_learn_vb_online::init fields (:761-783)
			rlog_out = new std::ofstream(r.rlog_file.c_str());
			if (!rlog_out->is_open()) throw std::string("Unable to open file " + r.rlog_file);
			std::cout << "logging to " << r.rlog_file << std::endl;
			rlog = new RLog(rlog_out);
			for (const char *f : {"rmse", "mae", "time_pred", "time_learn", "time_learn2", "time_learn4", "alpha",
			                      "rmse_mcmc_this", "rmse_mcmc_all"})
				rlog->add(f);
			for (uint32_t g = 0; g < r.G; g++) {
				std::ostringstream ss;
				ss << "wmu[" << g << "]"; rlog->add(ss.str()); ss.str("");
				ss << "wlambda[" << g << "]"; rlog->add(ss.str()); ss.str("");
				for (int f = 0; f < r.k; f++) {
					ss << "vmu[" << g << "," << f << "]"; rlog->add(ss.str()); ss.str("");
					ss << "vlambda[" << g << "," << f << "]"; rlog->add(ss.str()); ss.str("");
				}
			}
			rlog->init();
		}
		std::cout << "check in fm_learn_vb_online_simultaneous" << std::endl;
		std::ostringstream tag;
		tag << r.k0 << r.k1 << r.k;
		// :37-52: the rmse file and an (always empty) free_energy_..._vb_online are truncated; the
		// free energies are appended to free_energy_..._vb (fm_learn_vb_online.h:636-662)
		const std::string f_rmse = "test_rmse_" + tag.str() + "_vb_online", f_fe = "free_energy_" + tag.str() + "_vb";
		if (!resume) { std::ofstream a(f_rmse.c_str()); std::ofstream b(("free_energy_" + tag.str() + "_vb_online").c_str()); }
		ParityLog plog(r.parity_file, true);
		plog_setup(plog, ctx, "vb_online");
		for (uint32_t it = it0; it < it0 + r.num_iter; it++) {
			const double t_user = usertime();
			const clock_t t_clock = clock();
			const double t_wall = (double)time(NULL);
			vbfm_online_stats st;
			check(vbfm_online_epoch(ctx, &st), ctx);
			{
				std::ofstream fe(f_fe.c_str(), std::ios_base::app);
				fe << -st.free_energy_first << "\n";
				std::cout << "free energy " << st.free_energy_first << std::endl;
				if (r.num_batch > 1) {
					fe << -st.free_energy_last << "\n";
					std::cout << "free energy " << st.free_energy_last << std::endl;
				}
			}
			nan_reports(st.nan_alpha, st.inf_alpha, st.nan_mu_w, st.inf_mu_w, st.nan_sigma_w, st.nan_mu_v, st.inf_mu_v,
			            st.nan_sigma_v);
			if (rlog) {
				rlog->log("time_learn", usertime() - t_user);
				rlog->log("time_learn2", (double)(clock() - t_clock) / CLOCKS_PER_SEC);
				rlog->log("time_learn4", (double)time(NULL) - t_wall);
				rlog->log("rmse_mcmc_this", st.rmse);
				rlog->newline();
			}
			std::ofstream fr(f_rmse.c_str(), std::ios_base::app);
			fr << st.rmse << "\n";
			std::cout << "#Iter=" << std::setw(3) << it << "\tTest=" << st.rmse << std::endl;
			if (plog.on()) {
				plog.begin("vb_online", it);
				const double vals[] = {st.rmse, st.mae, st.free_energy_first, st.free_energy_last, st.alpha, st.sigma_0,
				                       st.mu_0_dash, st.sigma_0_dash, st.ms_regroup, st.ms_predict, st.ms_w0, st.ms_w,
				                       st.ms_v, st.ms_hyper, st.ms_test, st.ms_total};
				const char *keys[] = {"test_rmse", "test_mae", "free_energy_first", "free_energy_last", "alpha", "sigma_0",
				                      "mu_0_dash", "sigma_0_dash", "ms_regroup", "ms_predict", "ms_w0", "ms_w", "ms_v",
				                      "ms_hyper", "ms_test", "ms_total"};
				for (size_t i = 0; i < sizeof(vals) / sizeof(vals[0]); i++) plog.num(keys[i], vals[i]);
				plog.num("levels", st.num_levels);
				plog.num("level_launches", st.n_vlevel_launches);
				plog.num("sweep_nnz_k_per_s", st.ms_v > 0 ? (double)train.h.nnz * r.k / (st.ms_v * 1e-3) : NAN);
				plog.end();
			}
		}
		if (!r.save_file.empty()) check(vbfm_save_state(ctx, r.save_file.c_str(), it0 + r.num_iter), ctx);
		std::cout << "after learn" << std::endl;                              // libfm.cpp:507
		std::cout << "Final\tTrain=" << NAN << "\tTest=" << NAN << std::endl;   // evaluate() is NaN (:17)
		if (!r.out_file.empty()) {
			std::vector<double> pred(test.h.num_rows);
			check(vbfm_get_test_pred(ctx, pred.data()), ctx);
			std::ofstream o(r.out_file.c_str());
			for (double x : pred) o << x << std::endl;
		}
		delete rlog;
		delete rlog_out;
		vbfm_destroy(ctx);
	} catch (...) {
		if (ctx) vbfm_destroy(ctx);
		throw;
	}
}

// -method vb (libfm.cpp:306-311, 366, 496-519; fm_learn_vb_simultaneous.h:18-259)
struct VbRun {
	uint32_t seed;
	double init_stdev;
	uint32_t num_iter;
	const uint32_t *groups;
	uint32_t G, D;
	int k0, k1, k;
	bool vfile;
	std::string rlog_file, out_file, save_file, resume_file, parity_file;
};

static void run_vb(const VbRun &r, Data &train, Data &test, const Rank &rk)
{
	vbfm_ctx *ctx = nullptr;
	try {
		vbfm_config cfg{r.k0, r.k1, r.k, r.D, r.G, r.groups, train.h.min_target, train.h.max_target, rk.device, 0};
		check(vbfm_create(&ctx, &cfg), nullptr);
		join(ctx, rk);
		{
			const Slice tr = rk.slice(train.h), te = rk.slice(test.h);
			check(vbfm_set_train(ctx, &tr.csc), ctx);
			check(vbfm_set_test(ctx, &te.csc), ctx);
		}
		const int k = r.k;
		const uint32_t D = r.D, G = r.G;

		// fm.init + fm.w.init_normal + fml->init draws (libfm.cpp:123-366): the same stream on
		// the host (small models) or generated on the device (VBFM_INIT=host|replay overrides);
		// every rank draws the same values. -resume takes the state from its file instead (no
		// draws, no v_file.txt)
		const bool resume = !r.resume_file.empty();
		const size_t kd = (size_t)k * D;
		const bool vfile = r.vfile && !resume && rk.lead();
		const char *init_env = getenv("VBFM_INIT");
		const bool replay = init_env ? std::string(init_env) == "replay" : kd + D >= 2000000;
		std::vector<double> fm_v(vfile || (!replay && !resume) ? kd : 0);
		if (replay && !resume) {
			check(vbfm_init_params_replay(ctx, r.seed, r.init_stdev, vfile ? fm_v.data() : nullptr, nullptr), ctx);
		} else if (!resume) {
			std::vector<double> mu_w(D), sig_w(D), mu_v(kd), sig_v(kd), hw(G), hv((size_t)G * k);
			vbfm_params p{mu_w.data(), sig_w.data(), mu_v.data(), sig_v.data(), hw.data(), hv.data(), 0, 0, 0, 0};
			check(vbfm_init_params_host(r.seed, r.init_stdev, k, D, G, &p, fm_v.data(), nullptr), nullptr);
			check(vbfm_set_params(ctx, &p), ctx);
		}
		if (vfile) write_vfile(fm_v, k, D);
		fm_v.clear();
		fm_v.shrink_to_fit();

		// -rlog (libfm.cpp:353-363; fields of fm_learn::init and fm_learn_vb::init)
		std::ofstream *rlog_out = nullptr;
		RLog *rlog = nullptr;
		if (!r.rlog_file.empty() && rk.lead()) {
			rlog_out = new std::ofstream(r.rlog_file.c_str());
			if (!rlog_out->is_open()) throw std::string("Unable to open file " + r.rlog_file);
			std::cout << "logging to " << r.rlog_file << std::endl;
			rlog = new RLog(rlog_out);
			for (const char *f : {"rmse", "mae", "time_pred", "time_learn", "time_learn2", "time_learn4", "alpha",
			                      "rmse_mcmc_this", "rmse_mcmc_all"})
				rlog->add(f);
			for (uint32_t g = 0; g < G; g++) {
				std::ostringstream ss;
				ss << "wmu[" << g << "]"; rlog->add(ss.str()); ss.str("");
				ss << "wlambda[" << g << "]"; rlog->add(ss.str()); ss.str("");
				for (int f = 0; f < k; f++) {
					ss << "vmu[" << g << "," << f << "]"; rlog->add(ss.str()); ss.str("");
					ss << "vlambda[" << g << "," << f << "]"; rlog->add(ss.str()); ss.str("");
				}
			}
			rlog->init();
		}

		// fm_learn_vb_simultaneous::_learn
		uint32_t it0 = 0;
		if (resume) {
			check(vbfm_load_state(ctx, rk.rank_file(r.resume_file).c_str(), &it0), ctx);
			std::cout << "resuming from " << r.resume_file << " after " << it0 << " iterations" << std::endl;
		} else {
			check(vbfm_init_caches(ctx), ctx);
		}
		std::ostringstream tag;
		tag << r.k0 << r.k1 << k;
		const std::string f_rmse = "test_rmse_" + tag.str() + "_vb", f_fe = "free_energy_" + tag.str() + "_vb";
		if (!resume && rk.lead()) { std::ofstream a(f_rmse.c_str()); std::ofstream b(f_fe.c_str()); }   // truncate (:58-73); a resumed run appends
		ParityLog plog(r.parity_file, rk.lead());
		plog_setup(plog, ctx, "vb");
		for (uint32_t it = it0; it < it0 + r.num_iter; it++) {
			time_t now = time(0);
			std::cout << ctime(&now) << std::endl;
			const double t_user = usertime();
			const clock_t t_clock = clock();
			const double t_wall = (double)time(NULL);
			vbfm_iter_stats st;
			check(vbfm_iterate(ctx, &st), ctx);
			if (st.free_energy_valid) {   // fm_learn_vb.h:678-680
				if (rk.lead()) {
					std::ofstream fe(f_fe.c_str(), std::ios_base::app);
					fe << -st.free_energy << "\n";
				}
				std::cout << "free energy " << st.free_energy << std::endl;
			}
			nan_reports(st.nan_alpha, st.inf_alpha, st.nan_mu_w, st.inf_mu_w, st.nan_sigma_w, st.nan_mu_v, st.inf_mu_v,
			            st.nan_sigma_v);
			if (rlog) {
				rlog->log("time_learn", usertime() - t_user);
				rlog->log("time_learn2", (double)(clock() - t_clock) / CLOCKS_PER_SEC);
				rlog->log("time_learn4", (double)time(NULL) - t_wall);
				rlog->log("rmse_mcmc_this", st.rmse);
				rlog->newline();
			}
			if (rk.lead()) {
				std::ofstream fr(f_rmse.c_str(), std::ios_base::app);
				fr << st.rmse << "\n";
			}
			std::cout << "#Iter=" << std::setw(3) << it << "\tTrain=" << st.train_quirk << "\tTest=" << st.rmse << std::endl;
			if (plog.on()) {
				plog.begin("vb", it);
				const double vals[] = {st.train_quirk, st.rmse, st.mae, st.free_energy_valid ? st.free_energy : NAN, st.alpha,
				                       st.sigma_0, st.mu_0_dash, st.sigma_0_dash, st.ms_w0, st.ms_w, st.ms_qcache, st.ms_v,
				                       st.ms_hyper, st.ms_test, st.ms_total};
				const char *keys[] = {"train", "test_rmse", "test_mae", "free_energy", "alpha", "sigma_0", "mu_0_dash",
				                      "sigma_0_dash", "ms_w0", "ms_w", "ms_qcache", "ms_v", "ms_hyper", "ms_test", "ms_total"};
				for (size_t i = 0; i < sizeof(vals) / sizeof(vals[0]); i++) plog.num(keys[i], vals[i]);
				const uint32_t nans[] = {st.nan_mu_w, st.nan_sigma_w, st.inf_mu_w, st.nan_mu_v, st.nan_sigma_v, st.inf_mu_v,
				                         st.nan_alpha, st.inf_alpha};
				const char *nkeys[] = {"nan_mu_w", "nan_sigma_w", "inf_mu_w", "nan_mu_v", "nan_sigma_v", "inf_mu_v",
				                       "nan_alpha", "inf_alpha"};
				for (size_t i = 0; i < sizeof(nans) / sizeof(nans[0]); i++) plog.num(nkeys[i], nans[i]);
				plog.num("levels", st.num_levels);
				plog.sweep(st.ms_v, k, train.h.nnz, train.h.num_rows, train.h.num_feature, rk.nranks, false);
				plog.exchange(ctx);
				plog.end();
			}
		}
		if (!r.save_file.empty())
			check(vbfm_save_state(ctx, rk.rank_file(r.save_file).c_str(), it0 + r.num_iter), ctx);
		// libfm.cpp:509-511: fm_learn_vb::evaluate returns NaN
		std::cout << "Final\tTrain=" << NAN << "\tTest=" << NAN << std::endl;
		if (!r.out_file.empty()) {   // libfm.cpp:514-519, DVector::save (matrix.h:284-295)
			uint32_t lo, hi;
			rk.range(test.h.num_rows, &lo, &hi);
			std::vector<double> pred(hi - lo), all;
			check(vbfm_get_test_pred(ctx, pred.data()), ctx);
			gather_test(rk, test, pred, &all);
			if (rk.lead()) {
				std::ofstream o(r.out_file.c_str());
				for (double v : all) o << v << std::endl;
			}
		}
		delete rlog;
		delete rlog_out;
		vbfm_destroy(ctx);
	} catch (...) {
		if (ctx) vbfm_destroy(ctx);
		throw;
	}
}

// everything one rank runs, given the parsed command line
struct Job {
	std::string method;
	VbRun vb;
	McmcRun mc;
	OnlineRun online;
	bool plan = false;
};

// -plan 1: the rank's launch and shard plan as one JSON line; with -transport host the ranks
// also all-reduce their rank numbers through the shared slots (sum and max), so the exchange
// itself is exercised without a GPU
static void print_plan(const Job &job, const Data &train, const Data &test, const Rank &rk)
{
	const Slice tr = rk.slice(train.h), te = rk.slice(test.h);
	uint32_t lo, hi, tlo, thi;
	rk.range(train.h.num_rows, &lo, &hi);
	rk.range(test.h.num_rows, &tlo, &thi);
	double xs[2] = {(double)rk.rank, (double)tr.csc.nnz};
	uint32_t xm = (uint32_t)rk.rank;
	const bool xchg = rk.multi() && rk.host;
	if (xchg) {
		shm_exchange((void *)&rk, xs, 2, VBFM_X_F64, VBFM_X_SUM);
		shm_exchange((void *)&rk, &xm, 1, VBFM_X_U32, VBFM_X_MAX);
	}
	char line[1024];
	snprintf(line, sizeof(line),
	         "{\"rank\": %d, \"nranks\": %d, \"device\": %d, \"transport\": \"%s\", \"shard\": \"%s\", "
	         "\"method\": \"%s\", \"train_rows\": [%u, %u], \"train_nnz\": %llu, \"train_features\": %u, "
	         "\"test_rows\": [%u, %u], \"test_nnz\": %llu, \"xchg_rank_sum\": %.17g, \"xchg_nnz_sum\": %.17g, "
	         "\"xchg_rank_max\": %d}\n",
	         rk.rank, rk.nranks, rk.device, !rk.multi() ? "none" : rk.host ? "host" : "rccl",
	         rk.shard == VBFM_SHARD_ROWS ? "rows" : "features", job.method.c_str(), lo, hi,
	         (unsigned long long)tr.csc.nnz, tr.csc.num_feature, tlo, thi, (unsigned long long)te.csc.nnz,
	         xchg ? xs[0] : -1.0, xchg ? xs[1] : -1.0, xchg ? (int)xm : -1);
	fputs(line, stdout);
	fflush(stdout);
}

// one rank of the run. Returns the process exit status of a rank (0 ok).
static int run_rank(const Job &job, Data &train, Data &test, Rank &rk)
{
	try {
		if (job.plan) { print_plan(job, train, test, rk); return 0; }
		if (rk.device < 0) {   // -devices N -transport host: rank r on device r % visible
			int32_t n = 0;
			check(vbfm_device_count(&n), nullptr);
			if (n <= 0) throw std::string("no HIP device available");
			rk.device = rk.rank % n;
		}
		if (job.method == "vb_online") run_online(job.online, train, test, rk);
		else if (job.method == "vb") run_vb(job.vb, train, test, rk);
		else run_mcmc(job.mc, train, test, rk);
		return 0;
	} catch (std::string &e) {
		std::cerr << std::endl << "ERROR: " << (rk.multi() ? "rank " + std::to_string(rk.rank) + ": " : "") << e
		          << std::endl;
	} catch (char const *e) {
		std::cerr << std::endl << "ERROR: " << (rk.multi() ? "rank " + std::to_string(rk.rank) + ": " : "") << e
		          << std::endl;
	}
	return 1;
}

// Fork one process per rank (no HIP call has happened in this process), wait for them, kill the
// others when one fails (a rank left waiting at a barrier or inside a collective would never
// return). The shared page is mapped before the fork, so every rank sees the same one.
static int launch(const Job &job, Data &train, Data &test, Rank proto, const std::vector<int32_t> &ordinals)
{
	const int P = proto.nranks;
	const size_t slot = (size_t)4 << 20;   // 4 MB per rank and exchange chunk
	const size_t hdr = (sizeof(ShmHeader) + 4095) / 4096 * 4096;
	const size_t bytes = hdr + (size_t)P * slot + (size_t)test.h.num_rows * sizeof(double) + 4096;
	void *mem = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
	if (mem == MAP_FAILED) throw std::string("cannot map the ranks' shared page");
	ShmHeader *shm = (ShmHeader *)mem;
	pthread_barrierattr_t at;
	pthread_barrierattr_init(&at);
	pthread_barrierattr_setpshared(&at, PTHREAD_PROCESS_SHARED);
	if (pthread_barrier_init(&shm->bar, &at, (unsigned)P) != 0) throw std::string("cannot create the ranks' barrier");
	pthread_barrierattr_destroy(&at);
	shm->slot_bytes = slot;
	shm->nranks = P;
	proto.shm = shm;
	proto.slots = (char *)mem + hdr;
	proto.test_pred = (double *)(proto.slots + (size_t)P * slot);
	std::cout.flush();
	fflush(stdout);
	fflush(stderr);
	std::vector<pid_t> pids;
	for (int r = 0; r < P; r++) {
		const pid_t pid = fork();
		if (pid < 0) {
			for (pid_t q : pids) kill(q, SIGKILL);
			throw std::string("fork failed");
		}
		if (pid == 0) {
			Rank rk = proto;
			rk.rank = r;
			rk.device = ordinals.empty() ? (proto.host ? -1 : r) : ordinals[r];
			if (!rk.lead() && !job.plan) std::cout.setstate(std::ios::badbit);   // rank 0 speaks for the job
			const int rc = run_rank(job, train, test, rk);
			std::cout.flush();
			fflush(stdout);
			fflush(stderr);
			_exit(rc);
		}
		pids.push_back(pid);
	}
	int failed = -1, status_failed = 0;
	size_t left = pids.size();
	while (left > 0) {
		int status = 0;
		const pid_t pid = waitpid(-1, &status, 0);
		if (pid < 0) break;
		const auto it = std::find(pids.begin(), pids.end(), pid);
		if (it == pids.end()) continue;
		left--;
		const bool ok = WIFEXITED(status) && WEXITSTATUS(status) == 0;
		if (!ok && failed < 0) {
			failed = (int)(it - pids.begin());
			status_failed = status;
			for (pid_t q : pids)   // the ranks still running; a reaped one is 0 (never kill(-1 or 0, ...))
				if (q > 0 && q != pid) kill(q, SIGKILL);
		}
		*it = 0;
	}
	pthread_barrier_destroy(&shm->bar);
	munmap(mem, bytes);
	if (failed >= 0) {
		std::ostringstream m;
		m << "rank " << failed << " of " << P << " failed ("
		  << (WIFSIGNALED(status_failed) ? "signal " + std::to_string(WTERMSIG(status_failed))
		                                 : "exit status " + std::to_string(WEXITSTATUS(status_failed)))
		  << "); the other ranks were stopped";
		throw m.str();
	}
	return 0;
}

int main(int argc, char **argv)
{
	try {
		CmdLine cmd(argc, argv);
		std::cout << "----------------------------------------------------------------------------" << std::endl;
		std::cout << "libFM (VB learner on MI355X, libvbfm ABI " << vbfm_abi_version() << ")" << std::endl;
		std::cout << "  Version: 1.4.2 (reference CLI surface)" << std::endl;
		std::cout << "----------------------------------------------------------------------------" << std::endl;
		if (vbfm_abi_version() != VBFM_ABI_VERSION)
			throw std::string("libvbfm.so ABI " + std::to_string(vbfm_abi_version()) + " but this libFM was built for ABI " +
			                  std::to_string(VBFM_ABI_VERSION));
		const std::string p_task = cmd.reg("task", "r=regression, c=binary classification [MANDATORY]");
		const std::string p_meta = cmd.reg("meta", "filename for meta information about data set");
		const std::string p_train = cmd.reg("train", "filename for training data [MANDATORY]");
		const std::string p_test = cmd.reg("test", "filename for test data [MANDATORY]");
		cmd.reg("validation", "filename for validation data (only for SGDA)");
		const std::string p_out = cmd.reg("out", "filename for output");
		const std::string p_dim = cmd.reg("dim", "'k0,k1,k2': k0=use bias, k1=use 1-way interactions, k2=dim of 2-way interactions; default=1,1,8");
		const std::string p_reg = cmd.reg("regular", "'r0,r1,r2' for SGD and ALS: r0=bias regularization, r1=1-way regularization, r2=2-way regularization");
		const std::string p_init = cmd.reg("init_stdev", "stdev for initialization of 2-way factors; default=0.1");
		cmd.reg("stdev", "standard deviation for the model; default=1");
		const std::string p_iter = cmd.reg("iter", "number of iterations; default=100");
		cmd.reg("learn_rate", "learn_rate for SGD; default=0.1");
		const std::string p_method = cmd.reg("method", "learning method (SGD, SGDA, ALS, MCMC, VB); default=MCMC");
		const std::string p_verb = cmd.reg("verbosity", "how much infos to print; default=0");
		const std::string p_rlog = cmd.reg("rlog", "write measurements within iterations to a file; default=''");
		const std::string p_seed = cmd.reg("seed", "integer value, default=time(NULL)");
		const std::string p_help = cmd.reg("help", "this screen");
		const std::string p_rel = cmd.reg("relation", "BS: filenames for the relations, default=''");
		cmd.reg("cache_size", "cache size for data storage (only applicable if data is in binary format), default=infty");
		const std::string p_batch = cmd.reg("batch", "How many batches for online algorithm");
		const std::string p_dev = cmd.reg("device", "HIP device ordinal of a one-GPU run; default=0");
		const std::string p_devs = cmd.reg("devices", "GPUs: a count N (ranks on ordinals 0..N-1) or a list 'o0,o1,...' of ordinals, one rank each; default=1");
		const std::string p_shard = cmd.reg("shard", "partition over the ranks: rows (exact, default) or features (the columns of every level; Jacobi across ranks, vb only)");
		const std::string p_trans = cmd.reg("transport", "rank exchange: rccl (one GPU per rank, default) or host (shared memory; ranks may share a GPU)");
		const std::string p_plan = cmd.reg("plan", "1: every rank prints its launch and shard plan as JSON and exits (no GPU)");
		const std::string p_vfile = cmd.reg("vfile", "write v_file.txt like the reference (1) or not (0); default=1");
		const std::string p_save = cmd.reg("save_state", "vb, vb_online, mcmc, als: write the learner's state to this file after the last iteration (.<rank> per rank with -devices)");
		const std::string p_plog = cmd.reg("parity_log", "JSON lines: a 'setup' line (set-up costs), then one per iteration: the printed values at 17 digits, phase times, sweep nnz*k/s, HBM roofline fraction and the exchange's calls / bytes / ms; default=''");
		const std::string p_resume = cmd.reg("resume", "vb, vb_online, mcmc, als: continue from a -save_state file (same data and -dim) instead of the initial draws");
		if (cmd.has(p_help) || argc == 1) { cmd.print_help(); return 0; }
		cmd.check();

		const uint32_t seed = cmd.has(p_seed) ? (uint32_t)cmd.geti(p_seed, 0) : (uint32_t)time(NULL);
		const std::string method = cmd.get(p_method, "mcmc");
		if (method != "vb" && method != "vb_online" && method != "mcmc" && method != "als")
			throw std::string("method " + method + " is not provided by this build (use -method vb, vb_online, mcmc or als)");
		if (cmd.get(p_task) != "r") throw std::string("unknown task");   // regression only
		if (!cmd.list(p_rel).empty()) throw std::string("-relation is not supported by this build");

		// the ranks: -devices N | o0,o1,..., -shard, -transport (checked before the data load)
		Rank proto;
		std::vector<int32_t> ordinals;
		{
			const std::vector<std::string> devs = cmd.list(p_devs);
			if (devs.size() > 1) {
				for (const std::string &d : devs) ordinals.push_back((int32_t)atoi(d.c_str()));
				proto.nranks = (int32_t)ordinals.size();
			} else if (devs.size() == 1) {
				proto.nranks = (int32_t)atoi(devs[0].c_str());
			}
			if (proto.nranks < 1 || proto.nranks > 256) throw std::string("-devices: expected a rank count 1..256 or a list of ordinals");
			for (int32_t o : ordinals)
				if (o < 0) throw std::string("-devices: negative ordinal");
			const std::string tr = cmd.get(p_trans, "rccl"), sh = cmd.get(p_shard, "rows");
			if (tr != "rccl" && tr != "host") throw std::string("-transport: rccl or host");
			if (sh != "rows" && sh != "features") throw std::string("-shard: rows or features");
			proto.host = tr == "host";
			proto.shard = sh == "rows" ? VBFM_SHARD_ROWS : VBFM_SHARD_FEATURES;
			if (proto.shard == VBFM_SHARD_FEATURES && method != "vb")
				throw std::string("-shard features is a -method vb mode");
			if (proto.nranks > 1 && method == "vb_online") throw std::string("-method vb_online runs on one GPU (-devices 1)");
			if (!proto.host && !ordinals.empty()) {
				std::vector<int32_t> o = ordinals;
				std::sort(o.begin(), o.end());
				if (std::adjacent_find(o.begin(), o.end()) != o.end())
					throw std::string("-devices: RCCL needs one GPU per rank (-transport host lets ranks share one)");
			}
			proto.device = proto.nranks == 1 ? (ordinals.empty() ? (int32_t)cmd.geti(p_dev, 0) : ordinals[0]) : 0;
		}

		Data train, test;
		const double t_load = wall_now();
		load(cmd.get(p_train), train, "train");
		load(cmd.get(p_test), test, "test");
		g_load_s = wall_now() - t_load;
		if (cmd.geti(p_verb, 0) > 0) std::cout << "seed=" << seed << std::endl;
		if (proto.row_shards() && train.h.num_rows < (uint32_t)proto.nranks)
			throw std::string("-devices: fewer train rows than ranks");

		// libfm.cpp:215-256: attributes and groups. For vb_online the train file is only scanned
		// (find_max_feature, libfm.cpp:167-170, 528-600), which leaves the largest feature ids in
		// num_feature: one attribute fewer than -method vb gets on the same files
		const uint32_t nf_max = std::max(train.h.num_feature, test.h.num_feature);
		const uint32_t D = method == "vb_online" ? nf_max : nf_max + 1;
		std::vector<uint32_t> groups(D, 0);
		uint32_t G = 1;
		if (cmd.has(p_meta)) {
			std::ifstream in(cmd.get(p_meta));
			if (!in.is_open()) throw std::string("Unable to open file " + cmd.get(p_meta));
			G = 0;
			for (uint32_t i = 0; i < D; i++) {
				long g = 0;
				in >> g;
				groups[i] = (uint32_t)g;
				G = std::max(G, groups[i] + 1);
			}
		}
		// -dim (libfm.cpp:266-271)
		std::vector<std::string> dim = cmd.list(p_dim);
		if (dim.empty()) dim = {"1", "1", "8"};
		if (dim.size() != 3) throw std::string("-dim needs three values");
		const int k0 = atoi(dim[0].c_str()) != 0, k1 = atoi(dim[1].c_str()) != 0, k = atoi(dim[2].c_str());
		const double init_stdev = cmd.getd(p_init, 0.1);
		const uint32_t num_iter = (uint32_t)cmd.geti(p_iter, 100);
		const uint32_t *gp = cmd.has(p_meta) ? groups.data() : nullptr;
		const bool vfile = cmd.geti(p_vfile, 1) != 0;
		const std::string rlog = cmd.has(p_rlog) ? cmd.get(p_rlog) : std::string();
		const std::string out = cmd.has(p_out) ? cmd.get(p_out) : std::string();
		const std::string plog = cmd.has(p_plog) ? cmd.get(p_plog) : std::string();

		Job job;
		job.method = method;
		job.plan = cmd.geti(p_plan, 0) != 0;
		job.online = OnlineRun{seed, init_stdev, num_iter, (uint32_t)cmd.geti(p_batch, 50), gp, G, D, k0, k1, k, vfile,
		                       rlog, out, plog, cmd.has(p_save) ? cmd.get(p_save) : std::string(),
		                       cmd.has(p_resume) ? cmd.get(p_resume) : std::string()};
		std::vector<double> reg;
		for (const std::string &r : cmd.list(p_reg)) reg.push_back(atof(r.c_str()));
		job.mc = McmcRun{method == "mcmc", seed, init_stdev, num_iter, reg, gp, G, D, k0, k1, k, vfile, rlog, out, plog,
		                 cmd.has(p_save) ? cmd.get(p_save) : std::string(), cmd.has(p_resume) ? cmd.get(p_resume) : std::string()};
		job.vb = VbRun{seed, init_stdev, num_iter, gp, G, D, k0, k1, k, vfile, rlog, out,
		               cmd.has(p_save) ? cmd.get(p_save) : std::string(), cmd.has(p_resume) ? cmd.get(p_resume) : std::string(),
		               plog};

		if (proto.nranks == 1) {   // one GPU, this process
			run_rank(job, train, test, proto);
			return 0;
		}
		launch(job, train, test, proto, ordinals);
	} catch (std::string &e) {
		std::cerr << std::endl << "ERROR: " << e << std::endl;   // libfm.cpp:521-525 (exit code 0 there too)
	} catch (char const *e) {
		std::cerr << std::endl << "ERROR: " << e << std::endl;
	}
	return 0;
}
