// xflow-amd: `xflow_lr` native CLI, argument compatible with the reference
// binary (/root/reference/src/model/main.cc:15-48):
//     xflow_lr <train_prefix> <test_prefix> <model 0|1|2> <epochs>
// ps-lite roles come from DMLC_ROLE like the reference launch scripts: the
// scheduler and server roles have nothing to do here (every rank owns a shard
// of the HBM table) and exit after printing what the reference prints; a
// worker trains.  Multi-worker runs go through the Python launcher
// (python -m xflow_amd.cli, scripts/local.sh), which maps workers to GPUs.
// Optional flags after the positional args: --threads N --device D
// --serial-slices --keep-remainder --sgd --fm-standard --mvm-fixed
// --mvm-predict-compat --v-dim D --log2-cap N --save PATH --load PATH.
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

#include "xflow/trainer.h"

int main(int argc, char* argv[]) {
  if (argc < 5) {
    std::cout << "sh run_ps_local.sh model_index epochs\n";
    std::cout << "LR model expmple: sh run_ps_local.sh 0 100\n";
    std::cout << "FM model expmple: sh run_ps_local.sh 1 100\n";
    std::cout << std::endl;
    return 1;
  }
  const char* role = std::getenv("DMLC_ROLE");
  std::string r = role ? role : "worker";
  if (r == "server") {
    std::cout << "init server success " << std::endl;
    return 0;
  }
  if (r == "scheduler") return 0;

  xflow::TrainerConfig cfg;
  cfg.train_prefix = argv[1];
  cfg.test_prefix = argv[2];
  cfg.epochs = std::atoi(argv[4]);
  std::string save, load;
  const char* dev = std::getenv("XFLOW_DEVICE");
  const bool gpu = xflow::hip_backend_available();
  cfg.device = gpu ? (dev ? std::atoi(dev) : 0) : -1;
  for (int i = 5; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) {
        std::cerr << "missing value for " << a << std::endl;
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--threads") cfg.threads = std::atoi(next());
    else if (a == "--device") cfg.device = std::atoi(next());
    else if (a == "--serial-slices") cfg.serial_slices = true;
    else if (a == "--keep-remainder") cfg.keep_remainder = true;
    else if (a == "--sgd") cfg.opt.kind = xflow::kSGD;
    else if (a == "--fm-standard") cfg.model_spec.fm_math = xflow::kFmStandard;
    else if (a == "--mvm-fixed") cfg.model_spec.mvm_math = xflow::kMvmFixed;
    else if (a == "--mvm-predict-compat") cfg.mvm_predict_compat = true;
    else if (a == "--v-dim") cfg.model_spec.v_dim = std::atoi(next());
    else if (a == "--log2-cap") cfg.table_log2_cap = std::atoi(next());
    else if (a == "--train-block-bytes") cfg.train_block_bytes = std::atoll(next());
    else if (a == "--save") save = next();
    else if (a == "--load") load = next();
    else {
      std::cerr << "unknown flag " << a << std::endl;
      return 2;
    }
  }
  char m = argv[3][0];
  if (m == '0') {
    cfg.model = xflow::kLR;
    std::cout << "start LR " << std::endl;
  } else if (m == '1') {
    cfg.model = xflow::kFM;
    std::cout << "start FM " << std::endl;
  } else if (m == '2') {
    cfg.model = xflow::kMVM;
    std::cout << "start MVM " << std::endl;
  } else {
    std::cerr << "model must be 0 (LR), 1 (FM) or 2 (MVM)" << std::endl;
    return 2;
  }
  const char* rk = std::getenv("RANK");
  if (rk) cfg.rank = std::atoi(rk);
  try {
    xflow::Trainer t(cfg);
    if (!load.empty()) t.engine().load(load);
    t.train();
    if (!save.empty()) t.engine().save(save);
  } catch (const std::exception& e) {
    std::cerr << "xflow_lr: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
