// oracle/ref_binding.cpp -- TEST INFRASTRUCTURE ONLY: the reference-side binding of libvbfm.so,
// compiled and run (INTEGRATION.md §2 made real).
//
// This is the learner class a maintainer would add to the reference: it compiles against the
// UNMODIFIED reference headers straight from /root/reference/src (-I, nothing copied), plugs
// into the reference's learner seam (the abstract fm_learn, src/libfm/src/fm_learn.h:38-265)
// as a subclass of the reference's own fm_learn_vb_simultaneous, and replaces only its
// learn() (fm_learn_vb.h:746-786 + fm_learn_vb_simultaneous.h:18-259) by calls through the
// C-ABI (include/vbfm.h). Everything around it is reference code, in the order of the
// reference CLI's `-method vb` flow (src/libfm/libfm.cpp:123-366, 496-506):
//   srand(seed)                                   libfm.cpp:123-124 (the CLI uses time(NULL))
//   DataSubset::load of train and test            libfm.cpp:137-158 (the reference's loader,
//                                                 incl. create_data_t, Data.h:106-283,457-509)
//   num_all_attribute, DataMetaInfo               libfm.cpp:215-256
//   fm.init(), fm.w.init_normal                   libfm.cpp:259-274, 307
//   fml->init(): the reference's fm_learn_vb::init (priors, mu' draws on the same rand() stream)
//   fml->learn(train, test): HERE -- the reference's data_t / targets and its variational
//                                 arrays handed to libvbfm, the iterations on the GPU
// and prints the reference's "#Iter=" lines plus full-precision "BIND" lines that
// tests/test_ref_binding_gpu.py compares with the reference's own golden trace (sa_k8).
//
// Build: make -C oracle ref (needs /root/reference and lib/libvbfm.so); output oracle/_ref/.
#include <cstdlib>
#include <cstdio>
#include <iostream>
#include <string>
#include <iterator>
#include <algorithm>
#include <fstream>
#include <sstream>
#include <vector>
#include <iomanip>
#include "util/util.h"
#include "util/cmdline.h"
#include "fm_core/fm_model.h"
#include "libfm/src/Data.h"
#include "libfm/src/fm_learn.h"
#include "libfm/src/fm_learn_mcmc_simultaneous.h"   // e_q_term, relation_cache (as libfm.cpp's include order)
#include "libfm/src/fm_learn_vb_simultaneous.h"
#include "vbfm.h"

// the reference's learner with its learn() running on the MI355X through libvbfm.so
class fm_learn_vb_hip : public fm_learn_vb_simultaneous {
public:
	int device = 0;
	vbfm_ctx* ctx = NULL;

	~fm_learn_vb_hip() { if (ctx) vbfm_destroy(ctx); }

	virtual void learn(DataSubset& train, DataSubset& test) {
		const uint D = fm->num_attribute, k = fm->num_factor, G = meta->num_attr_groups;
		std::vector<uint32_t> group(D);
		for (uint j = 0; j < D; j++) group[j] = meta->attr_group(j);
		vbfm_config cfg = {fm->k0 ? 1 : 0, fm->k1 ? 1 : 0, (int32_t)k, D, G, group.data(),
		                   (float)min_target, (float)max_target, device, task};
		check(vbfm_create(&ctx, &cfg), "vbfm_create");
		// the reference's transposed data (data_t, Data::create_data_t) and targets
		std::vector<uint64_t> cp_tr, cp_te;
		std::vector<vbfm_entry> ent_tr, ent_te;
		std::vector<float> y_tr, y_te;
		vbfm_csc tr = csc_of(train, cp_tr, ent_tr, y_tr), te = csc_of(test, cp_te, ent_te, y_te);
		check(vbfm_set_train(ctx, &tr), "vbfm_set_train");
		check(vbfm_set_test(ctx, &te), "vbfm_set_test");
		// the variational / hyper parameters fm_learn_vb::init drew (fm_learn_vb.h:685-743)
		std::vector<double> mv((size_t)k * D), sv((size_t)k * D), hv((size_t)G * k);
		for (uint f = 0; f < k; f++)
			for (uint j = 0; j < D; j++) {
				mv[(size_t)f * D + j] = mu_v_dash(f, j);
				sv[(size_t)f * D + j] = sigma_v_dash(f, j);
			}
		for (uint g = 0; g < G; g++)
			for (uint f = 0; f < k; f++) hv[(size_t)g * k + f] = sigma_v(g, f);
		vbfm_params p = {mu_w_dash.value, sigma_w_dash.value, mv.data(), sv.data(), sigma_w.value, hv.data(),
		                 alpha, sigma_0, mu_0_dash, sigma_0_dash};
		check(vbfm_set_params(ctx, &p), "vbfm_set_params");
		check(vbfm_init_caches(ctx), "vbfm_init_caches");   // fm_learn_vb_simultaneous.h:37-44
		for (uint i = 0; i < num_iter; i++) {
			vbfm_iter_stats st;
			check(vbfm_iterate(ctx, &st), "vbfm_iterate");
			std::cout << "#Iter=" << std::setw(3) << i << "\tTrain=" << st.train_quirk << "\tTest=" << st.rmse
			          << std::endl;
			std::ostringstream b;
			b.precision(17);
			b << "BIND " << i << " rmse " << st.rmse << " mae " << st.mae << " train " << st.train_quirk
			  << " free_energy " << st.free_energy << " alpha " << st.alpha << " levels " << st.num_levels;
			std::cout << b.str() << std::endl;
		}
		// results back into the reference's own members (as its learner leaves them)
		check(vbfm_get_params(ctx, &p), "vbfm_get_params");
		for (uint f = 0; f < k; f++)
			for (uint j = 0; j < D; j++) {
				mu_v_dash(f, j) = mv[(size_t)f * D + j];
				sigma_v_dash(f, j) = sv[(size_t)f * D + j];
			}
		for (uint g = 0; g < G; g++)
			for (uint f = 0; f < k; f++) sigma_v(g, f) = hv[(size_t)g * k + f];
		alpha = p.alpha; sigma_0 = p.sigma_0; mu_0_dash = p.mu_0_dash; sigma_0_dash = p.sigma_0_dash;
		pred_this.setSize(test.num_cases);
		check(vbfm_get_test_pred(ctx, pred_this.value), "vbfm_get_test_pred");
	}

	double sum_mu_w() { double s = 0; for (uint j = 0; j < mu_w_dash.dim; j++) s += mu_w_dash(j); return s; }
	double sq_mu_w() { double s = 0; for (uint j = 0; j < mu_w_dash.dim; j++) s += mu_w_dash(j) * mu_w_dash(j); return s; }

private:
	void check(int rc, const char* what) {
		if (rc) throw std::string(what) + ": " + vbfm_last_error(ctx);
	}
	// data_t row j = feature j's entries (ascending rows); vbfm_entry == sparse_entry<float>
	static vbfm_csc csc_of(DataSubset& d, std::vector<uint64_t>& cp, std::vector<vbfm_entry>& ent,
	                       std::vector<float>& y) {
		LargeSparseMatrix<DATA_FLOAT>* t = d.data_t;
		if (t == NULL) throw std::string("the data set has no transposed copy (data_t)");
		const uint nf = t->getNumRows();
		cp.assign(nf + 1, 0);
		ent.clear();
		ent.reserve(t->getNumValues());
		for (t->begin(); !t->end(); t->next()) {
			sparse_row<DATA_FLOAT>& r = t->getRow();
			for (uint i = 0; i < r.size; i++) ent.push_back(vbfm_entry{r.data[i].id, (float)r.data[i].value});
			cp[t->getRowIndex() + 1] = ent.size();
		}
		for (uint j = 0; j < nf; j++) if (cp[j + 1] < cp[j]) cp[j + 1] = cp[j];
		y.resize(d.num_cases);
		for (uint c = 0; c < d.num_cases; c++) y[c] = (float)d.target(c);
		vbfm_csc c = {d.num_cases, nf, ent.size(), cp.data(), ent.data(), y.data()};
		return c;
	}
};

static std::string arg(int argc, char** argv, const char* name, const char* dflt) {
	for (int i = 1; i + 1 < argc; i++) if (std::string(argv[i]) == name) return argv[i + 1];
	return dflt;
}

int main(int argc, char** argv) {
	std::cout.precision(17);
	try {
		std::string train_f = arg(argc, argv, "--train", ""), test_f = arg(argc, argv, "--test", "");
		std::string dim = arg(argc, argv, "--dim", "1,1,8");
		uint num_iter = atoi(arg(argc, argv, "--iter", "20").c_str());
		long seed = atol(arg(argc, argv, "--seed", "1").c_str());
		double init_stdev = atof(arg(argc, argv, "--init_stdev", "0.1").c_str());
		srand(seed);                                            // libfm.cpp:123-124
		DataSubset train(0, true, true), test(0, true, true);    // libfm.cpp:137-158
		train.load(train_f);
		test.load(test_f);
		uint num_all_attribute = std::max(train.num_feature, test.num_feature) + 1;   // libfm.cpp:215
		DataMetaInfo meta(num_all_attribute);
		meta.num_relations = 0;
		fm_model fm;                                             // libfm.cpp:259-274
		fm.num_attribute = num_all_attribute;
		fm.init_stdev = init_stdev;
		{
			std::vector<int> d;
			std::stringstream ss(dim);
			std::string tok;
			while (std::getline(ss, tok, ',')) d.push_back(atoi(tok.c_str()));
			fm.k0 = d[0] != 0; fm.k1 = d[1] != 0; fm.num_factor = d[2];
		}
		fm.init();
		fm.w.init_normal(fm.init_mean, fm.init_stdev);          // libfm.cpp:307
		fm_learn_vb_hip* fml = new fm_learn_vb_hip();
		fml->num_iter = num_iter;
		fml->num_eval_cases = test.num_cases;
		fml->validation = NULL;
		fml->fm = &fm;                                           // libfm.cpp:331-366
		fml->max_target = train.max_target;
		fml->min_target = train.min_target;
		fml->meta = &meta;
		fml->task = 0;
		fml->log = NULL;
		fml->device = atoi(arg(argc, argv, "--device", "0").c_str());
		fml->init();
		fml->learn(train, test);                                 // libfm.cpp:496-506
		std::cout << "BIND_FINAL sum_mu_w " << fml->sum_mu_w() << " sq_mu_w " << fml->sq_mu_w() << " mu_0_dash "
		          << fml->mu_0_dash << " alpha " << fml->alpha << std::endl;
		delete fml;
	} catch (std::string& e) {
		std::cerr << "ERROR: " << e << std::endl;
		return 1;
	} catch (char const* e) {
		std::cerr << "ERROR: " << e << std::endl;
		return 1;
	}
	return 0;
}
