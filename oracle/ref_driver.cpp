// oracle/ref_driver.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).
//
// A driver that compiles the UNMODIFIED reference headers straight from
// /root/reference/src (passed with -I by oracle/Makefile; nothing is copied) and
// runs the reference's own fm_learn_vb code with a fixed seed, dumping its state at
// full precision so the C restatement (oracle/vbfm_oracle.c) and the HIP path can be
// pinned against it.
//
// The setup mirrors the reference CLI's `-method vb` flow, in the same RNG order:
//   srand(seed)                                   src/libfm/libfm.cpp:123-124 (CLI uses time(NULL))
//   DataSubset(cache 0, has_x, has_xt) + load     src/libfm/libfm.cpp:137-158
//   num_all_attribute = max(nf_train,nf_test)+1   src/libfm/libfm.cpp:215
//   DataMetaInfo (+ optional -meta groups)        src/libfm/libfm.cpp:219-256
//   fm.init()  (v ~ N(0,init_stdev), v_file.txt)  src/libfm/libfm.cpp:259-274, src/fm_core/fm_model.h:92-101
//   fm.w.init_normal(0, init_stdev)               src/libfm/libfm.cpp:307
//   fml->init()                                   src/libfm/libfm.cpp:366, src/libfm/src/fm_learn_vb.h:685-743
// and the iteration loop restates fm_learn_vb_simultaneous::_learn
// (src/libfm/src/fm_learn_vb_simultaneous.h:18-259) around the reference's own protected
// step methods, so every number comes from reference code.
//
// Modes (all write raw little-endian arrays into --dump DIR):
//   vb      : full VB run, per-iteration trace (trace.txt) and parameter dumps.
//   steps   : one pass of the update_all sweep step by step (fm_learn_vb.h:383-440) with
//             cache dumps after each step.
//   levels  : the same sweeps with each dependency level's features in turn (ascending ids
//             inside a level) and cache / parameter dumps after every level (the per-level
//             parity of vbfm_step_w_level / vbfm_step_v_level).
//   sweep   : CPU-baseline timing of the factor sweep (add_main_q + update_v over all
//             features, fm_learn_vb.h:409-440) on a loaded data set; prints one JSON line.
//   als/mcmc: MCMC/ALS learner (fm_learn_mcmc_simultaneous.h:50-305), per-iteration trace.
//   vb_online: the reference's own fm_learn_vb_online_simultaneous (OVBFM, -method vb_online)
//             with the data setup of libfm.cpp:159-171 (train never loaded, find_max_feature,
//             libfm.cpp:528-600, restated below); it writes its batch files next to --train, so
//             callers pass a private copy. "#Iter=" / "free energy" lines + final parameters.

#include <cstdlib>
#include <cstdio>
#include <iostream>
#include <string>
#include <iterator>
#include <algorithm>
#include <iomanip>
#include <fstream>
#include <sstream>
#include <vector>
#include <chrono>
#include "util/util.h"
#include "util/cmdline.h"
#include "fm_core/fm_model.h"
#include "libfm/src/Data.h"
#include "libfm/src/fm_learn.h"
#include "libfm/src/fm_learn_mcmc_simultaneous.h"
#include "libfm/src/fm_learn_vb_simultaneous.h"
#include "libfm/src/fm_learn_vb_online_simultaneous.h"

static std::string g_dump;

static void dump_arr(const std::string& name, const double* p, size_t n) {
	if (g_dump.empty()) return;
	std::string fn = g_dump + "/" + name + ".f64";
	FILE* f = fopen(fn.c_str(), "wb");
	if (!f) { fprintf(stderr, "cannot write %s\n", fn.c_str()); exit(3); }
	fwrite(p, sizeof(double), n, f);
	fclose(f);
}

static double now_s() {
	return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

class RefVB : public fm_learn_vb_simultaneous {
public:
	std::string mode;
	uint sweep_factors;
	FILE* trace;

	void dump_rows(const std::string& tag, DataSubset& train) {
		uint n = train.num_cases;
		std::vector<double> e(n), t(n), q(n), tq(n), tz(n);
		for (uint i = 0; i < n; i++) {
			e[i] = cache[i].e; q[i] = cache[i].q;
			t[i] = cache_t[i].t; tq[i] = cache_t[i].q; tz[i] = cache_t[i].z;
		}
		dump_arr(tag + "_e", e.data(), n);
		dump_arr(tag + "_t", t.data(), n);
		dump_arr(tag + "_q", q.data(), n);
		dump_arr(tag + "_tq", tq.data(), n);
		dump_arr(tag + "_tz", tz.data(), n);
	}
	void dump_params(const std::string& tag) {
		dump_arr(tag + "_mu_w", mu_w_dash.value, mu_w_dash.dim);
		dump_arr(tag + "_sigma_w", sigma_w_dash.value, sigma_w_dash.dim);
		dump_arr(tag + "_mu_v", mu_v_dash.value[0], (size_t)mu_v_dash.dim1 * mu_v_dash.dim2);
		dump_arr(tag + "_sigma_v", sigma_v_dash.value[0], (size_t)sigma_v_dash.dim1 * sigma_v_dash.dim2);
		dump_arr(tag + "_hyp_sigma_w", sigma_w.value, sigma_w.dim);
		if (sigma_v.dim1 * sigma_v.dim2 > 0)
			dump_arr(tag + "_hyp_sigma_v", sigma_v.value[0], (size_t)sigma_v.dim1 * sigma_v.dim2);
		double sc[6] = {alpha, sigma_0, mu_0_dash, sigma_0_dash, 0, 0};
		dump_arr(tag + "_scalars", sc, 6);
	}

	void init_caches(DataSubset& train, DataSubset& test) {
		DVector<DataSubset*> main_data(2);
		DVector<e_q_term*> main_cache(2);
		main_data(0) = &train; main_data(1) = &test;
		main_cache(0) = cache; main_cache(1) = cache_test;
		predict_data_and_write_to_eterms(main_data, main_cache);
		predict_t_and_write_to_qterms(&train, cache_t);
		for (uint c = 0; c < train.num_cases; c++) cache[c].e = train.target(c) - cache[c].e;
	}

	virtual void _learn(DataSubset& train, DataSubset& test) {
		if (mode == "steps") { run_steps(train, test); return; }
		if (mode == "levels") { run_levels(train, test); return; }
		if (mode == "sweep") { run_sweep(train); return; }
		run_vb(train, test);
	}

	// restatement of the loop in fm_learn_vb_simultaneous.h:75-258 (regression only)
	void run_vb(DataSubset& train, DataSubset& test) {
		init_caches(train, test);
		{
			std::vector<double> te(test.num_cases);
			for (uint c = 0; c < test.num_cases; c++) te[c] = cache_test[c].e;
			dump_arr("init_test_e", te.data(), te.size());
			dump_rows("init", train);
		}
		DVector<DataSubset*> only_test(1);
		DVector<e_q_term*> only_test_cache(1);
		only_test(0) = &test; only_test_cache(0) = cache_test;
		for (uint it = 0; it < num_iter; it++) {
			std::cout << "ITER_BEGIN " << it << std::endl;
			update_all(train);     // prints "free energy <F>" (17 digits: cout precision set in main)
			predict_data_and_write_to_eterms(only_test, only_test_cache);
			for (uint c = 0; c < test.num_cases; c++) {
				double p = cache_test[c].e;
				p = std::min(max_target, p);
				p = std::max(min_target, p);
				pred_this(c) = p;
			}
			double rmse_train = 0.0;
			for (uint c = 0; c < train.num_cases; c++) {
				double p = cache[c].e;
				p = std::min(max_target, p);
				p = std::max(min_target, p);
				rmse_train += p * p;
			}
			rmse_train = std::sqrt(rmse_train / train.num_cases);
			double rmse, mae;
			_evaluate(pred_this, test.target, 1.0, rmse, mae, num_eval_cases);
			double s_mu_w = 0, s_mu_v = 0, s_sig_w = 0, s_sig_v = 0;
			for (uint i = 0; i < mu_w_dash.dim; i++) { s_mu_w += mu_w_dash(i) * mu_w_dash(i); s_sig_w += sigma_w_dash(i); }
			for (uint f = 0; f < mu_v_dash.dim1; f++)
				for (uint i = 0; i < mu_v_dash.dim2; i++) { s_mu_v += mu_v_dash(f, i) * mu_v_dash(f, i); s_sig_v += sigma_v_dash(f, i); }
			std::cout << "ITER " << it << " rmse " << rmse << " mae " << mae << " train " << rmse_train
				<< " alpha " << alpha << " sigma_0 " << sigma_0 << " mu_0_dash " << mu_0_dash
				<< " sigma_0_dash " << sigma_0_dash << " sq_mu_w " << s_mu_w << " sum_sigma_w " << s_sig_w
				<< " sq_mu_v " << s_mu_v << " sum_sigma_v " << s_sig_v
				<< " nan_mu_v " << nan_mu_v_dash << " nan_sigma_v " << nan_sigma_v_dash
				<< " nan_mu_w " << nan_mu_w_dash << " nan_sigma_w " << nan_sigma_w_dash
				<< " nan_alpha " << nan_alpha << " inf_alpha " << inf_alpha << std::endl;
			std::ostringstream tag; tag << "iter" << it;
			if (getenv("REF_DUMP_ITER_PARAMS")) {
				dump_params(tag.str());
				std::vector<double> pt(test.num_cases);
				for (uint c = 0; c < test.num_cases; c++) pt[c] = pred_this(c);
				dump_arr(tag.str() + "_pred", pt.data(), pt.size());
				dump_rows(tag.str(), train);
			}
		}
		dump_params("final");
	}

	// update_all (fm_learn_vb.h:383-440) driven step by step through the reference's
	// own update_w0 / update_w / add_main_q / update_v methods.
	void run_steps(DataSubset& train, DataSubset& test) {
		init_caches(train, test);
		dump_rows("s0_init", train);
		{
			std::vector<double> te(test.num_cases);
			for (uint c = 0; c < test.num_cases; c++) te[c] = cache_test[c].e;
			dump_arr("s0_init_test_e", te.data(), te.size());
		}
		dump_params("s0");
		if (fm->k0) { update_w0(train); }
		dump_rows("s1_w0", train);
		dump_params("s1");
		if (fm->k1) {
			for (uint i = 0; i < train.data_t->getNumRows(); i++) {
				uint g = meta->attr_group(i);
				update_w(mu_w_dash(i), sigma_w_dash(i), sigma_w(g), train.data_t->getRow(i));
			}
		}
		dump_rows("s2_w", train);
		dump_params("s2");
		for (int f = 0; f < fm->num_factor; f++) {
			for (uint c = 0; c < train.num_cases; c++) { cache[c].q = 0.0; cache_t[c].q = 0.0; cache_t[c].z = 0.0; }
			add_main_q(train, f);
			std::ostringstream a; a << "s3_f" << f << "_q";
			dump_rows(a.str(), train);
			double* v = mu_v_dash.value[f];
			double* v1 = sigma_v_dash.value[f];
			for (uint i = 0; i < train.data_t->getNumRows(); i++) {
				uint g = meta->attr_group(i);
				update_v(f, v[i], v1[i], sigma_v(g, f), train.data_t->getRow(i));
			}
			std::ostringstream b; b << "s4_f" << f << "_v";
			dump_rows(b.str(), train);
			dump_params(b.str());
		}
		std::cout << "STEPS_DONE" << std::endl;
	}

	// Dependency level of every train feature: level(j) = 1 + max level of a
	// smaller feature id sharing a row with j, 1 without one -- the least fixed point of
	// level[b] >= level[a] + 1 over consecutive distinct ids a < b of every row (read from the
	// reference's own CSR, train.data).
	std::vector<uint> feature_levels(DataSubset& train) {
		const uint nf = train.data_t->getNumRows();
		std::vector<std::pair<uint, uint> > edges;
		for (train.data->begin(); !train.data->end(); train.data->next()) {
			sparse_row<DATA_FLOAT>& row = train.data->getRow();
			std::vector<uint> ids;
			for (uint i = 0; i < row.size; i++) ids.push_back(row.data[i].id);
			std::sort(ids.begin(), ids.end());
			ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
			for (size_t i = 1; i < ids.size(); i++) edges.push_back(std::make_pair(ids[i - 1], ids[i]));
		}
		std::vector<uint> level(nf, 1);
		for (bool changed = true; changed;) {
			changed = false;
			for (size_t e = 0; e < edges.size(); e++)
				if (level[edges[e].second] < level[edges[e].first] + 1) {
					level[edges[e].second] = level[edges[e].first] + 1;
					changed = true;
				}
		}
		return level;
	}

	// update_all's sweeps (fm_learn_vb.h:383-440) through the reference's own update_w /
	// add_main_q / update_v, the features of each dependency level in ascending id order, level
	// after level, with the caches and parameters dumped after every level. Features of
	// different levels commute where the ascending sweep interleaves them (no shared row), so
	// the state after the last level is the ascending sweep's bit for bit (checked against
	// the "steps" dumps by tests/test_oracle_golden.py); after level l it is what the GPU's
	// level kernels must hold after their level l (vbfm_step_w_level / vbfm_step_v_level).
	void run_levels(DataSubset& train, DataSubset& test) {
		init_caches(train, test);
		const std::vector<uint> level = feature_levels(train);
		uint L = 0;
		for (size_t j = 0; j < level.size(); j++) L = std::max(L, level[j]);
		std::cout << "LEVELS " << L << std::endl;
		std::vector<double> lv(level.begin(), level.end());
		dump_arr("levels", lv.data(), lv.size());
		if (fm->k0) update_w0(train);
		dump_rows("l_w0", train);
		const uint nf = train.data_t->getNumRows();
		if (fm->k1) {
			for (uint l = 1; l <= L; l++) {
				for (uint i = 0; i < nf; i++)
					if (level[i] == l) update_w(mu_w_dash(i), sigma_w_dash(i), sigma_w(meta->attr_group(i)), train.data_t->getRow(i));
				std::ostringstream a; a << "l_w_l" << (l - 1);
				dump_rows(a.str(), train);
				dump_params(a.str());
			}
		}
		for (int f = 0; f < fm->num_factor; f++) {
			for (uint c = 0; c < train.num_cases; c++) { cache[c].q = 0.0; cache_t[c].q = 0.0; cache_t[c].z = 0.0; }
			add_main_q(train, f);
			double* v = mu_v_dash.value[f];
			double* v1 = sigma_v_dash.value[f];
			for (uint l = 1; l <= L; l++) {
				for (uint i = 0; i < nf; i++)
					if (level[i] == l) update_v(f, v[i], v1[i], sigma_v(meta->attr_group(i), f), train.data_t->getRow(i));
				std::ostringstream a; a << "l_f" << f << "_l" << (l - 1);
				dump_rows(a.str(), train);
				dump_params(a.str());
			}
		}
		std::cout << "LEVELS_DONE" << std::endl;
	}

	// CPU baseline: time the factor sweep exactly as update_all runs it (fm_learn_vb.h:409-440).
	void run_sweep(DataSubset& train) {
		DVector<DataSubset*> main_data(1);
		DVector<e_q_term*> main_cache(1);
		main_data(0) = &train; main_cache(0) = cache;
		double t0 = now_s();
		predict_data_and_write_to_eterms(main_data, main_cache);
		predict_t_and_write_to_qterms(&train, cache_t);
		for (uint c = 0; c < train.num_cases; c++) cache[c].e = train.target(c) - cache[c].e;
		double t1 = now_s();
		// the k = 0 overhead of one iteration (fm_learn_vb.h:384-406): update_w0 + the w sweep
		if (fm->k0) update_w0(train);
		if (fm->k1)
			for (uint i = 0; i < train.data_t->getNumRows(); i++)
				update_w(mu_w_dash(i), sigma_w_dash(i), sigma_w(meta->attr_group(i)), train.data_t->getRow(i));
		double tw = now_s();
		const double init_s = t1 - t0, k0_s = tw - t1;
		t1 = tw;
		uint nf = std::min((uint)fm->num_factor, sweep_factors);
		for (uint f = 0; f < nf; f++) {
			for (uint c = 0; c < train.num_cases; c++) { cache[c].q = 0.0; cache_t[c].q = 0.0; cache_t[c].z = 0.0; }
			add_main_q(train, f);
			double* v = mu_v_dash.value[f];
			double* v1 = sigma_v_dash.value[f];
			for (uint i = 0; i < train.data_t->getNumRows(); i++) {
				uint g = meta->attr_group(i);
				update_v((int&)f, v[i], v1[i], sigma_v(g, f), train.data_t->getRow(i));
			}
		}
		double t2 = now_s();
		double s = 0;
		for (uint c = 0; c < train.num_cases; c++) s += cache[c].e;
		uint64 nnz = train.data_t->getNumValues();
		printf("{\"nnz\": %llu, \"rows\": %u, \"factors\": %u, \"init_s\": %.6f, \"k0_s\": %.6f, "
		       "\"sweep_s\": %.6f, \"nnz_k_per_s\": %.6e, \"checksum_e\": %.17g}\n",
		       (unsigned long long)nnz, train.num_cases, nf, init_s, k0_s, t2 - t1,
		       (double)nnz * nf / (t2 - t1), s);
	}
};

class RefOVB : public fm_learn_vb_online_simultaneous {
public:
	void dump_params(const std::string& tag) {
		dump_arr(tag + "_mu_w", mu_w_dash.value, mu_w_dash.dim);
		dump_arr(tag + "_sigma_w", sigma_w_dash.value, sigma_w_dash.dim);
		dump_arr(tag + "_mu_v", mu_v_dash.value[0], (size_t)mu_v_dash.dim1 * mu_v_dash.dim2);
		dump_arr(tag + "_sigma_v", sigma_v_dash.value[0], (size_t)sigma_v_dash.dim1 * sigma_v_dash.dim2);
		dump_arr(tag + "_hyp_sigma_w", sigma_w.value, sigma_w.dim);
		if (sigma_v.dim1 * sigma_v.dim2 > 0)
			dump_arr(tag + "_hyp_sigma_v", sigma_v.value[0], (size_t)sigma_v.dim1 * sigma_v.dim2);
		dump_arr(tag + "_nat_mu_w", natural_mu_w_dash.value, natural_mu_w_dash.dim);
		dump_arr(tag + "_nat_sigma_w", natural_sigma_w_dash.value, natural_sigma_w_dash.dim);
		dump_arr(tag + "_nat_mu_v", natural_mu_v_dash.value[0], (size_t)natural_mu_v_dash.dim1 * natural_mu_v_dash.dim2);
		dump_arr(tag + "_nat_sigma_v", natural_sigma_v_dash.value[0],
		         (size_t)natural_sigma_v_dash.dim1 * natural_sigma_v_dash.dim2);
		std::vector<double> steps;
		for (uint i = 0; i < new_wj.dim; i++) steps.push_back(new_wj(i));
		for (uint i = 0; i < new_vj.dim; i++) steps.push_back(new_vj(i));
		dump_arr(tag + "_steps", steps.data(), steps.size());
		double sc[8] = {alpha, sigma_0, mu_0_dash, sigma_0_dash, natural_mu_0_dash, natural_sigma_0_dash, new_w0, (double)t_w0};
		dump_arr(tag + "_scalars", sc, 8);
		dump_arr(tag + "_pred", pred_this.value, pred_this.dim);
	}
};

// find_max_feature (libfm.cpp:528-600): counts, largest feature ids and targets of the text files
static void max_feature_of(const std::string& fn, DataSubset& d) {
	std::ifstream f(fn.c_str());
	d.num_cases = 0;
	d.num_feature = 0;
	d.min_target = +std::numeric_limits<DATA_FLOAT>::max();
	d.max_target = -std::numeric_limits<DATA_FLOAT>::max();
	while (!f.eof()) {
		int nchar;
		float rating;
		uint feature;
		double value;
		std::string line;
		std::getline(f, line);
		const char* pline = line.c_str();
		while ((*pline == ' ') || (*pline == 9)) pline++;
		if ((*pline == 0) || (*pline == '#')) continue;
		if (sscanf(pline, "%f%n", &rating, &nchar) >= 1) {
			d.min_target = std::min(rating, d.min_target);
			d.max_target = std::max(rating, d.max_target);
			pline += nchar;
			while (sscanf(pline, "%u:%lf%n", &feature, &value, &nchar) >= 2) {
				pline += nchar;
				d.num_feature = std::max(feature, (uint)d.num_feature);
			}
		} else {
			throw "cannot parse line \"" + line + "\"";
		}
		d.num_cases++;
	}
}

class RefMCMC : public fm_learn_mcmc_simultaneous {
	// as the reference, trace lines come from _learn's "#Iter=" output at 17 digits
};

static std::string arg(int argc, char** argv, const std::string& key, const std::string& def) {
	for (int i = 2; i + 1 < argc; i++) if (key == argv[i]) return argv[i + 1];
	return def;
}

int main(int argc, char** argv) {
	if (argc < 2) {
		fprintf(stderr, "usage: ref_driver vb|steps|levels|sweep|als|mcmc --train F --test F --dim k0,k1,k --iter N --seed S [--init_stdev x] [--meta F] [--regular r0,rw,rv] [--dump DIR] [--sweep_factors n]\n");
		return 2;
	}
	std::cout.precision(17);
	try {
		std::string mode = argv[1];
		std::string train_f = arg(argc, argv, "--train", "");
		std::string test_f = arg(argc, argv, "--test", "");
		std::string dim = arg(argc, argv, "--dim", "1,1,8");
		uint num_iter = atoi(arg(argc, argv, "--iter", "1").c_str());
		long seed = atol(arg(argc, argv, "--seed", "1").c_str());
		double init_stdev = atof(arg(argc, argv, "--init_stdev", "0.1").c_str());
		std::string meta_f = arg(argc, argv, "--meta", "");
		g_dump = arg(argc, argv, "--dump", "");
		uint sweep_factors = atoi(arg(argc, argv, "--sweep_factors", "1000000").c_str());

		srand(seed);
		bool is_mcmc = (mode == "als" || mode == "mcmc");
		bool is_online = (mode == "vb_online");
		DataSubset train(0, !is_mcmc, true);
		DataSubset test(0, !is_mcmc, true);
		if (is_online) {   // libfm.cpp:159-171
			test.load(test_f);
			max_feature_of(train_f, train);
			max_feature_of(test_f, test);
		} else {
			train.load(train_f);
			test.load(test_f);
		}
		uint num_all_attribute = std::max(train.num_feature, test.num_feature) + 1;
		DataMetaInfo meta_main(num_all_attribute);
		if (!meta_f.empty()) meta_main.loadGroupsFromFile(meta_f);
		DataMetaInfo meta(num_all_attribute);
		meta.num_attr_groups = meta_main.num_attr_groups;
		meta.num_attr_per_group.setSize(meta.num_attr_groups);
		meta.num_attr_per_group.init(0);
		for (uint i = 0; i < meta_main.attr_group.dim; i++) {
			meta.attr_group(i) = meta_main.attr_group(i);
			meta.num_attr_per_group(meta.attr_group(i))++;
		}
		meta.num_relations = 0;

		fm_model fm;
		fm.num_attribute = num_all_attribute;
		fm.init_stdev = init_stdev;
		fm.stdev = 1.0;
		{
			std::vector<int> d;
			std::stringstream ss(dim);
			std::string tok;
			while (std::getline(ss, tok, ',')) d.push_back(atoi(tok.c_str()));
			fm.k0 = d[0] != 0; fm.k1 = d[1] != 0; fm.num_factor = d[2]; fm.num_factor_new = d[2];
		}
		fm.init();
		std::cout << "NUMS train_rows " << train.num_cases << " train_nf " << train.num_feature
			<< " test_rows " << test.num_cases << " test_nf " << test.num_feature
			<< " D " << num_all_attribute << " min_target " << train.min_target
			<< " max_target " << train.max_target << std::endl;
		dump_arr("init_fm_v", fm.v.value[0], (size_t)fm.v.dim1 * fm.v.dim2);

		fm.w.init_normal(fm.init_mean, fm.init_stdev);
		dump_arr("init_fm_w", fm.w.value, fm.w.dim);
		fm_learn* fml;
		RefVB* vb = NULL;
		RefOVB* ovb = NULL;
		if (is_online) {   // libfm.cpp:312-320
			ovb = new RefOVB();
			ovb->num_iter = num_iter;
			ovb->num_eval_cases = test.num_cases;
			ovb->training_file = train_f;
			ovb->testing_file = test_f;
			ovb->num_batch = atoi(arg(argc, argv, "--batch", "50").c_str());
			fml = ovb;
		} else if (is_mcmc) {
			RefMCMC* m = new RefMCMC();
			m->num_iter = num_iter;
			m->num_eval_cases = test.num_cases;
			m->do_sample = (mode == "mcmc");
			m->do_multilevel = (mode == "mcmc");
			fml = m;
		} else {
			vb = new RefVB();
			vb->mode = mode;
			vb->sweep_factors = sweep_factors;
			vb->num_iter = num_iter;
			vb->num_eval_cases = test.num_cases;
			fml = vb;
		}
		fml->validation = NULL;
		fml->fm = &fm;
		fml->max_target = train.max_target;
		fml->min_target = train.min_target;
		fml->meta = &meta;
		fml->task = 0;
		fml->log = NULL;
		fml->init();
		if (is_mcmc) {
			// -regular as libfm.cpp:367-411 (absent => all zero)
			std::vector<double> reg;
			{
				std::stringstream ss(arg(argc, argv, "--regular", ""));
				std::string tok;
				while (std::getline(ss, tok, ',')) if (!tok.empty()) reg.push_back(atof(tok.c_str()));
			}
			fm_learn_mcmc* m = (fm_learn_mcmc*)fml;
			if (reg.size() == 0) { fm.reg0 = 0.0; fm.regw = 0.0; fm.regv = 0.0; }
			else if (reg.size() == 1) { fm.reg0 = reg[0]; fm.regw = reg[0]; fm.regv = reg[0]; }
			else if (reg.size() == 3) { fm.reg0 = reg[0]; fm.regw = reg[1]; fm.regv = reg[2]; }
			if (reg.size() == 1 + 2 * (size_t)meta.num_attr_groups && reg.size() != 3 && reg.size() != 1) {
				fm.reg0 = reg[0]; fm.regw = 0.0; fm.regv = 0.0;
				size_t j = 1;
				for (uint g = 0; g < meta.num_attr_groups; g++) m->w_lambda(g) = reg[j++];
				for (uint g = 0; g < meta.num_attr_groups; g++) {
					for (int f = 0; f < fm.num_factor; f++) m->v_lambda(g, f) = reg[j];
					j++;
				}
			} else {
				m->w_lambda.init(fm.regw);
				m->v_lambda.init(fm.regv);
			}
		} else if (ovb) {
			ovb->dump_params("init");   // pred_this is not sized yet: an empty dump
		} else {
			vb->dump_params("init");
		}
		fml->learn(train, test);
		if (ovb) {
			ovb->dump_params("final");
		}
		if (is_mcmc) {
			fm_learn_mcmc* m = (fm_learn_mcmc*)fml;
			dump_arr("final_fm_v", fm.v.value[0], (size_t)fm.v.dim1 * fm.v.dim2);
			dump_arr("final_fm_w", fm.w.value, fm.w.dim);
			double sc[2] = {fm.w0, m->alpha};
			dump_arr("final_mcmc_scalars", sc, 2);
			dump_arr("final_w_mu", m->w_mu.value, m->w_mu.dim);
			dump_arr("final_w_lambda", m->w_lambda.value, m->w_lambda.dim);
			if (fm.num_factor > 0) {
				dump_arr("final_v_mu", m->v_mu.value[0], (size_t)m->v_mu.dim1 * m->v_mu.dim2);
				dump_arr("final_v_lambda", m->v_lambda.value[0], (size_t)m->v_lambda.dim1 * m->v_lambda.dim2);
			}
		}
		std::cout << "DONE" << std::endl;
	} catch (std::string& e) {
		std::cerr << "ERROR: " << e << std::endl;
		return 1;
	} catch (char const*& e) {
		std::cerr << "ERROR: " << e << std::endl;
		return 1;
	}
	return 0;
}
