/*
 * xflow-amd C API -- symbol-compatible with the reference's declared (but
 * unbuildable) src/c_api/c_api.h:26-29 (XFCreate / XFStartTrain), fixed to
 * return status codes, plus explicit configuration and teardown entry points.
 */
#ifndef XFLOW_AMD_C_API_H_
#define XFLOW_AMD_C_API_H_

#ifdef __cplusplus
#define XF_EXTERN_C extern "C"
#else
#define XF_EXTERN_C
#endif

#define XF_DLL XF_EXTERN_C __attribute__((visibility("default")))

/* Create an LR trainer over <train>-%05d / <test>-%05d shards (rank 0).
 * Returns 0 on success, -1 on error (see XFGetLastError). */
XF_DLL int XFCreate(void** h, const char* train_path, const char* test_path);
/* Run the full reference training: epochs, then rank-0 predict + AUC line. */
XF_DLL int XFStartTrain(void** h);

/* Extensions (not in the reference). */
XF_DLL int XFCreateEx(void** h, const char* train_path, const char* test_path, int model,
                      int epochs, int threads, int device);
XF_DLL int XFSetEpochs(void** h, int epochs);
XF_DLL int XFPredict(void** h, double* logloss_printed, double* auc);
XF_DLL int XFSave(void** h, const char* path);
XF_DLL int XFLoad(void** h, const char* path);
XF_DLL int XFFree(void** h);
XF_DLL const char* XFGetLastError(void);

#endif /* XFLOW_AMD_C_API_H_ */
