/* N-API addon over the libblsgpu C ABI (include/blsgpu.h): the binding a Lodestar maintainer loads from
 * packages/beacon-node/src/chain/bls/gpu/ (INTEGRATION.md).  It only marshals: every input array is
 * copied by blsgpu_submit() before it returns, so JS may reuse its buffers as soon as submit() returns
 * (the reference structured-clones the same data, multithread/index.ts:157-164).  Completion runs on a
 * runtime thread and is bridged to the JS main thread with a napi_threadsafe_function, where the Promise
 * resolves (or rejects on a call-level failure: a device error never becomes `false`,
 * multithread/index.ts:368-375).
 *
 * Exports:
 *   init(devices: number[] | null) -> ctx (external)             blsgpu_init
 *   close(ctx)                                                    blsgpu_destroy  (IBlsVerifier.close)
 *   deviceCount(ctx) -> number                                    blsgpu_device_count
 *   uploadPubkeys(ctx, firstIndex, Uint8Array 96*n)               blsgpu_pubkeys_upload (index2pubkey)
 *   pubkeysCount(ctx) -> number                                   blsgpu_pubkeys_count
 *   setOption(ctx, key, value)                                    blsgpu_set_option
 *   codeName(code) -> string                                      blsgpu_code_name
 *   submit(ctx, req) -> Promise<{results: Int8Array, groups, batchRetries, batchSigsSuccess, deviceMs, ...,
 *                                 urgentLane}>
 *     req = {jobFirstSet: Uint32Array, jobFlags?: Uint8Array (BLSGPU_JOB_BATCHABLE 1 | BLSGPU_JOB_URGENT 2),
 *            pkBytes?: Uint8Array,
 *            setPkFirst?: Uint32Array, pkIndex?: Uint32Array, msgs: Uint8Array, sigs: Uint8Array,
 *            sigLen: Uint32Array, sigStride: number, seed?: number}              blsgpu_submit
 *     (pkBytes alone: one 96-B key per set; pkBytes + setPkFirst: bytes-aggregate; setPkFirst + pkIndex:
 *      device table)
 *   keyValidate(ctx, Uint8Array, pkLen) -> {pk96, status}        blsgpu_key_validate (synchronous)
 *   debugInject(what, skip, count)                                blsgpu_debug_inject (only with BLSGPU_FAULT_INJECTION=1)
 */
#define NAPI_VERSION 6
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "blsgpu.h"

#define CHECK(env, call)                                                   \
  do {                                                                     \
    if ((call) != napi_ok) {                                               \
      napi_throw_error((env), NULL, "blsgpu_napi: N-API call failed: " #call); \
      return NULL;                                                         \
    }                                                                      \
  } while (0)

typedef struct {
  blsgpu_ctx* ctx;
} CtxBox;

typedef struct {
  int8_t* results;
  uint32_t n_jobs;
  blsgpu_stats stats;
  int status;
  napi_deferred deferred;
  napi_threadsafe_function tsfn;
} Call;

static napi_value throw_code(napi_env env, const char* what, int rc) {
  char msg[160];
  const char* name = blsgpu_code_name(rc);
  snprintf(msg, sizeof msg, "%s: %s", what, name ? name : "unknown blsgpu error");
  napi_throw_error(env, name, msg);
  return NULL;
}

static void ctx_finalize(napi_env env, void* data, void* hint) {
  (void)env;
  (void)hint;
  CtxBox* box = (CtxBox*)data;
  if (box->ctx) blsgpu_destroy(box->ctx);
  free(box);
}

static CtxBox* get_box(napi_env env, napi_value v) {
  void* p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, NULL, "blsgpu_napi: expected a context from init()");
    return NULL;
  }
  return (CtxBox*)p;
}

static CtxBox* get_open_box(napi_env env, napi_value v) {
  CtxBox* box = get_box(env, v);
  if (box && !box->ctx) {
    throw_code(env, "blsgpu", BLSGPU_ERR_CLOSED);
    return NULL;
  }
  return box;
}

static napi_value Init(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int devs[64];
  int n = 0;
  if (argc >= 1) {
    bool is_arr = false;
    napi_is_array(env, argv[0], &is_arr);
    if (is_arr) {
      uint32_t len = 0;
      CHECK(env, napi_get_array_length(env, argv[0], &len));
      for (uint32_t i = 0; i < len && n < 64; i++) {
        napi_value e;
        CHECK(env, napi_get_element(env, argv[0], i, &e));
        int32_t d;
        CHECK(env, napi_get_value_int32(env, e, &d));
        devs[n++] = d;
      }
    }
  }
  blsgpu_ctx* ctx = NULL;
  int rc = blsgpu_init(n ? devs : NULL, n, &ctx);
  if (rc != BLSGPU_OK) return throw_code(env, "blsgpu_init", rc);
  CtxBox* box = (CtxBox*)calloc(1, sizeof(CtxBox));
  box->ctx = ctx;
  napi_value out;
  CHECK(env, napi_create_external(env, box, ctx_finalize, NULL, &out));
  return out;
}

static napi_value Close(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  CtxBox* box = get_box(env, argv[0]);
  if (!box) return NULL;
  if (box->ctx) {
    /* waits for in-flight submissions (their callbacks are queued on the tsfn), fails queued ones */
    blsgpu_destroy(box->ctx);
    box->ctx = NULL;
  }
  return NULL;
}

static napi_value DeviceCount(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  CtxBox* box = get_open_box(env, argv[0]);
  if (!box) return NULL;
  napi_value out;
  CHECK(env, napi_create_int32(env, blsgpu_device_count(box->ctx), &out));
  return out;
}

static int get_typed(napi_env env, napi_value obj, const char* key, napi_typedarray_type want, void** data,
                     size_t* len, int required) {
  bool has = false;
  *data = NULL;
  *len = 0;
  if (napi_has_named_property(env, obj, key, &has) != napi_ok || !has) return required ? -1 : 0;
  napi_value v;
  napi_get_named_property(env, obj, key, &v);
  napi_valuetype t;
  napi_typeof(env, v, &t);
  if (t == napi_undefined || t == napi_null) return required ? -1 : 0;
  bool is_ta = false;
  napi_is_typedarray(env, v, &is_ta);
  if (!is_ta) return -1;
  napi_typedarray_type type;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &type, len, data, &ab, &off) != napi_ok) return -1;
  if (type != want) return -1;
  return 1;
}

static napi_value UploadPubkeys(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  CtxBox* box = get_open_box(env, argv[0]);
  if (!box) return NULL;
  uint32_t first;
  CHECK(env, napi_get_value_uint32(env, argv[1], &first));
  napi_typedarray_type type;
  size_t len;
  void* data;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, argv[2], &type, &len, &data, &ab, &off) != napi_ok || type != napi_uint8_array ||
      len % 96) {
    napi_throw_type_error(env, NULL, "uploadPubkeys: expected a Uint8Array of 96-byte uncompressed pubkeys");
    return NULL;
  }
  int rc = blsgpu_pubkeys_upload(box->ctx, first, (const uint8_t*)data, (uint32_t)(len / 96));
  if (rc != BLSGPU_OK) return throw_code(env, "uploadPubkeys", rc);
  return NULL;
}

static napi_value PubkeysCount(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  CtxBox* box = get_open_box(env, argv[0]);
  if (!box) return NULL;
  napi_value out;
  CHECK(env, napi_create_uint32(env, blsgpu_pubkeys_count(box->ctx), &out));
  return out;
}

static napi_value SetOption(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  CtxBox* box = get_open_box(env, argv[0]);
  if (!box) return NULL;
  char key[64];
  size_t kl;
  CHECK(env, napi_get_value_string_utf8(env, argv[1], key, sizeof key, &kl));
  int64_t value;
  CHECK(env, napi_get_value_int64(env, argv[2], &value));
  int rc = blsgpu_set_option(box->ctx, key, value);
  if (rc != BLSGPU_OK) return throw_code(env, "setOption", rc);
  return NULL;
}

static napi_value GetOption(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  CtxBox* box = get_open_box(env, argv[0]);
  if (!box) return NULL;
  char key[64];
  size_t kl;
  CHECK(env, napi_get_value_string_utf8(env, argv[1], key, sizeof key, &kl));
  int64_t value = 0;
  int rc = blsgpu_get_option(box->ctx, key, &value);
  if (rc != BLSGPU_OK) return throw_code(env, "getOption", rc);
  napi_value out;
  CHECK(env, napi_create_int64(env, value, &out));
  return out;
}

static napi_value CodeName(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int32_t code;
  CHECK(env, napi_get_value_int32(env, argv[0], &code));
  const char* name = blsgpu_code_name(code);
  napi_value out;
  if (!name) {
    CHECK(env, napi_get_null(env, &out));
  } else {
    CHECK(env, napi_create_string_utf8(env, name, NAPI_AUTO_LENGTH, &out));
  }
  return out;
}

/* runtime thread */
static void on_done(void* user, int status) {
  Call* c = (Call*)user;
  c->status = status;
  napi_call_threadsafe_function(c->tsfn, c, napi_tsfn_blocking);
}

static void set_num(napi_env env, napi_value obj, const char* key, double v) {
  napi_value x;
  napi_create_double(env, v, &x);
  napi_set_named_property(env, obj, key, x);
}

/* JS main thread */
static void settle_on_main(napi_env env, napi_value js_cb, void* context, void* data) {
  (void)js_cb;
  (void)context;
  Call* c = (Call*)data;
  if (env != NULL) {
    if (c->status != BLSGPU_OK) {
      const char* name = blsgpu_code_name(c->status);
      napi_value msg, code, err;
      napi_create_string_utf8(env, name ? name : "BLSGPU_DEVICE_ERROR", NAPI_AUTO_LENGTH, &msg);
      napi_create_string_utf8(env, name ? name : "BLSGPU_DEVICE_ERROR", NAPI_AUTO_LENGTH, &code);
      napi_create_error(env, code, msg, &err);
      napi_reject_deferred(env, c->deferred, err);
    } else {
      napi_value out, ab, arr;
      void* dst;
      napi_create_object(env, &out);
      napi_create_arraybuffer(env, c->n_jobs, &dst, &ab);
      if (c->n_jobs) memcpy(dst, c->results, c->n_jobs);
      napi_create_typedarray(env, napi_int8_array, c->n_jobs, ab, 0, &arr);
      napi_set_named_property(env, out, "results", arr);
      set_num(env, out, "groups", c->stats.groups);
      set_num(env, out, "batchRetries", c->stats.batch_retries);
      set_num(env, out, "batchSigsSuccess", c->stats.batch_sigs_success);
      set_num(env, out, "devicesUsed", c->stats.devices_used);
      set_num(env, out, "deviceMs", c->stats.device_ms);
      set_num(env, out, "uniqueMessages", c->stats.unique_messages);
      set_num(env, out, "pairingUnits", c->stats.pairing_units);
      set_num(env, out, "urgentLane", c->stats.urgent_lane);
      napi_resolve_deferred(env, c->deferred, out);
    }
  }
  napi_release_threadsafe_function(c->tsfn, napi_tsfn_release);
  free(c->results);
  free(c);
}

static napi_value Submit(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 2) {
    napi_throw_type_error(env, NULL, "submit(ctx, req)");
    return NULL;
  }
  CtxBox* box = get_open_box(env, argv[0]);
  if (!box) return NULL;
  napi_value req = argv[1];
  void *jfs, *flags, *pkb, *spf, *pki, *msgs, *sigs, *slen;
  size_t n_jfs, n_flags, n_pkb, n_spf, n_pki, n_msgs, n_sigs, n_slen;
  if (get_typed(env, req, "jobFirstSet", napi_uint32_array, &jfs, &n_jfs, 1) < 0 || n_jfs < 1 ||
      get_typed(env, req, "jobFlags", napi_uint8_array, &flags, &n_flags, 0) < 0 ||
      get_typed(env, req, "pkBytes", napi_uint8_array, &pkb, &n_pkb, 0) < 0 ||
      get_typed(env, req, "setPkFirst", napi_uint32_array, &spf, &n_spf, 0) < 0 ||
      get_typed(env, req, "pkIndex", napi_uint32_array, &pki, &n_pki, 0) < 0 ||
      get_typed(env, req, "msgs", napi_uint8_array, &msgs, &n_msgs, 1) < 0 ||
      get_typed(env, req, "sigs", napi_uint8_array, &sigs, &n_sigs, 1) < 0 ||
      get_typed(env, req, "sigLen", napi_uint32_array, &slen, &n_slen, 1) < 0) {
    napi_throw_type_error(env, NULL, "submit: malformed request (typed arrays expected)");
    return NULL;
  }
  uint32_t stride = 192;
  napi_value v;
  bool has = false;
  if (napi_has_named_property(env, req, "sigStride", &has) == napi_ok && has) {
    napi_get_named_property(env, req, "sigStride", &v);
    napi_get_value_uint32(env, v, &stride);
  }
  double seed_d = 0;
  if (napi_has_named_property(env, req, "seed", &has) == napi_ok && has) {
    napi_get_named_property(env, req, "seed", &v);
    napi_get_value_double(env, v, &seed_d);
  }
  uint32_t n_jobs = (uint32_t)n_jfs - 1, n_sets = (uint32_t)n_slen;
  /* shape checks on the host before anything reaches the device */
  int ok = ((const uint32_t*)jfs)[n_jobs] == n_sets && n_msgs == 32ull * n_sets &&
           n_sigs >= (size_t)stride * n_sets && (!flags || n_flags == n_jobs);
  if (pkb && !spf) ok = ok && n_pkb == 96ull * n_sets;  /* one key per set */
  else if (pkb) ok = ok && n_spf == n_sets + 1ull && 96ull * ((const uint32_t*)spf)[n_sets] <= n_pkb;  /* bytes aggregate */
  else ok = ok && spf && n_spf == n_sets + 1ull && ((const uint32_t*)spf)[n_sets] <= n_pki;  /* device table */
  if (!ok) {
    napi_throw_range_error(env, "BLSGPU_ERR_ARGS", "submit: inconsistent array sizes");
    return NULL;
  }
  blsgpu_batch b;
  memset(&b, 0, sizeof b);
  b.n_sets = n_sets;
  b.n_jobs = n_jobs;
  b.job_first_set = (const uint32_t*)jfs;
  b.job_flags = (const uint8_t*)flags;
  b.pk_bytes = (const uint8_t*)pkb;
  b.set_pk_first = (const uint32_t*)spf;
  b.pk_index = (const uint32_t*)pki;
  b.msgs = (const uint8_t*)msgs;
  b.sigs = (const uint8_t*)sigs;
  b.sig_len = (const uint32_t*)slen;
  b.sig_stride = stride;
  b.seed = (uint64_t)seed_d; /* 0 = OS CSPRNG scalars (production) */

  Call* c = (Call*)calloc(1, sizeof(Call));
  c->n_jobs = n_jobs;
  c->results = (int8_t*)calloc(n_jobs ? n_jobs : 1, 1);
  napi_value promise, name;
  CHECK(env, napi_create_promise(env, &c->deferred, &promise));
  CHECK(env, napi_create_string_utf8(env, "blsgpu_submit", NAPI_AUTO_LENGTH, &name));
  CHECK(env, napi_create_threadsafe_function(env, NULL, NULL, name, 0, 1, NULL, NULL, NULL, settle_on_main,
                                             &c->tsfn));
  int rc = blsgpu_submit(box->ctx, &b, c->results, &c->stats, on_done, c);
  if (rc != BLSGPU_OK) {
    /* nothing was queued: settle synchronously through the same path */
    c->status = rc;
    settle_on_main(env, NULL, NULL, c);
  }
  return promise;
}

/* keyValidate(ctx, Uint8Array pks, pkLen 48|96) -> {pk96: Uint8Array, status: Int8Array}  (synchronous) */
static napi_value KeyValidate(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 3) {
    napi_throw_type_error(env, NULL, "keyValidate(ctx, pks, pkLen)");
    return NULL;
  }
  CtxBox* box = get_open_box(env, argv[0]);
  if (!box) return NULL;
  napi_typedarray_type t;
  size_t len = 0;
  void* data = NULL;
  if (napi_get_typedarray_info(env, argv[1], &t, &len, &data, NULL, NULL) != napi_ok || t != napi_uint8_array) {
    napi_throw_type_error(env, NULL, "keyValidate: pks must be a Uint8Array");
    return NULL;
  }
  uint32_t pk_len = 0;
  napi_get_value_uint32(env, argv[2], &pk_len);
  if ((pk_len != 48 && pk_len != 96) || len % pk_len) {
    napi_throw_range_error(env, "BLSGPU_ERR_ARGS", "keyValidate: pkLen must be 48 or 96 and divide the input");
    return NULL;
  }
  uint32_t n = (uint32_t)(len / pk_len);
  napi_value ab_pk, ab_st, pk96, st, out;
  void *p_pk = NULL, *p_st = NULL;
  CHECK(env, napi_create_arraybuffer(env, 96 * (size_t)n, &p_pk, &ab_pk));
  CHECK(env, napi_create_arraybuffer(env, n ? n : 1, &p_st, &ab_st));
  int rc = blsgpu_key_validate(box->ctx, n, (const uint8_t*)data, pk_len, pk_len, (uint8_t*)p_pk, (int8_t*)p_st);
  if (rc != BLSGPU_OK) return throw_code(env, "blsgpu_key_validate", rc);
  CHECK(env, napi_create_typedarray(env, napi_uint8_array, 96 * (size_t)n, ab_pk, 0, &pk96));
  CHECK(env, napi_create_typedarray(env, napi_int8_array, n, ab_st, 0, &st));
  CHECK(env, napi_create_object(env, &out));
  napi_set_named_property(env, out, "pk96", pk96);
  napi_set_named_property(env, out, "status", st);
  return out;
}

/* debugInject(what, skip, count): blsgpu_debug_inject (test hook; BLSGPU_INJECT_ENTROPY 1, BLSGPU_INJECT_DEVICE 2) */
static napi_value DebugInject(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 3) {
    napi_throw_type_error(env, NULL, "debugInject(what, skip, count)");
    return NULL;
  }
  int32_t what = 0;
  int64_t skip = 0, count = 0;
  napi_get_value_int32(env, argv[0], &what);
  napi_get_value_int64(env, argv[1], &skip);
  napi_get_value_int64(env, argv[2], &count);
  int rc = blsgpu_debug_inject(what, skip, count);
  if (rc != BLSGPU_OK) return throw_code(env, "blsgpu_debug_inject", rc);
  return NULL;
}

static napi_value ModuleInit(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"init", NULL, Init, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"close", NULL, Close, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"deviceCount", NULL, DeviceCount, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"uploadPubkeys", NULL, UploadPubkeys, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"pubkeysCount", NULL, PubkeysCount, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"setOption", NULL, SetOption, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"getOption", NULL, GetOption, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"codeName", NULL, CodeName, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"submit", NULL, Submit, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"keyValidate", NULL, KeyValidate, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
  };
  napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
  /* the fault-injection test hook is exported, by its own definition, only to processes started with
   * BLSGPU_FAULT_INJECTION=1 (the library refuses to arm it otherwise) */
  const char* fi = getenv("BLSGPU_FAULT_INJECTION");
  if (fi && fi[0] == '1' && fi[1] == 0) {
    napi_property_descriptor inject = {"debugInject", NULL, DebugInject, NULL, NULL, NULL,
                                       (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable),
                                       NULL};
    napi_define_properties(env, exports, 1, &inject);
  }
  napi_value v;
  napi_create_int32(env, BLSGPU_ABI_VERSION, &v);
  napi_set_named_property(env, exports, "abiVersion", v);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, ModuleInit)
