// xflow-amd C API implementation (see c_api.h).  Reference:
// /root/reference/src/c_api/c_api.{h,cc} -- XFCreate wraps an LR worker,
// XFStartTrain runs train().  Here the handle owns a native Trainer; the
// device is the first GPU when one is visible, else the CPU backend.
#include "c_api.h"

#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>

#include "xflow/trainer.h"

namespace {

thread_local std::string g_last_error;

struct XFlow {
  xflow::TrainerConfig cfg;
  std::unique_ptr<xflow::Trainer> trainer;
  xflow::Trainer& get() {
    if (!trainer) trainer.reset(new xflow::Trainer(cfg));
    return *trainer;
  }
};

int default_device() {
  if (!xflow::hip_backend_available()) return -1;
  const char* e = std::getenv("XFLOW_DEVICE");
  return e ? std::atoi(e) : 0;
}

template <typename F>
int guarded(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_last_error = e.what();
  } catch (...) {
    g_last_error = "unknown error";
  }
  return -1;
}

XFlow* handle(void** h) {
  if (!h || !*h) throw std::invalid_argument("null xflow handle");
  return reinterpret_cast<XFlow*>(*h);
}

}  // namespace

XF_DLL int XFCreateEx(void** h, const char* train, const char* test, int model, int epochs,
                      int threads, int device) {
  return guarded([&] {
    if (!h || !train || !test) throw std::invalid_argument("XFCreate: null argument");
    XFlow* xf = new XFlow();
    xf->cfg.train_prefix = train;
    xf->cfg.test_prefix = test;
    xf->cfg.model = model;
    xf->cfg.epochs = epochs;
    xf->cfg.threads = threads;
    xf->cfg.device = device;
    *h = xf;
  });
}

XF_DLL int XFCreate(void** h, const char* train, const char* test) {
  return XFCreateEx(h, train, test, xflow::kLR, 60, 0, default_device());
}

XF_DLL int XFSetEpochs(void** h, int epochs) {
  return guarded([&] {
    XFlow* xf = handle(h);
    xf->cfg.epochs = epochs;
    if (xf->trainer) throw std::logic_error("XFSetEpochs: trainer already started");
  });
}

XF_DLL int XFStartTrain(void** h) {
  return guarded([&] { handle(h)->get().train(); });
}

XF_DLL int XFPredict(void** h, double* logloss, double* auc) {
  return guarded([&] {
    xflow::EvalResult r = handle(h)->get().predict(0);
    if (logloss) *logloss = r.logloss_printed;
    if (auc) *auc = r.auc;
  });
}

XF_DLL int XFSave(void** h, const char* path) {
  return guarded([&] { handle(h)->get().engine().save(path); });
}

XF_DLL int XFLoad(void** h, const char* path) {
  return guarded([&] { handle(h)->get().engine().load(path); });
}

XF_DLL int XFFree(void** h) {
  return guarded([&] {
    if (h && *h) {
      delete reinterpret_cast<XFlow*>(*h);
      *h = nullptr;
    }
  });
}

XF_DLL const char* XFGetLastError(void) { return g_last_error.c_str(); }
