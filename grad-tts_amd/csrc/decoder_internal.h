// Accessors of the decoder's parameter registry for the training-path host code (train_bwd.cpp); defined in
// decoder.cpp. Raw parameters: fp32, reference layouts, contiguous in state_dict inventory order.
#pragma once
#include <stdint.h>

#include <string>

#include "gradtts.h"

int gt_internal_layout(gt_decoder* d);         // raw-block offsets only (host; no device memory)
int gt_internal_prepare_raw(gt_decoder* d);    // layout + upload of the raw parameter block
const float* gt_internal_param(gt_decoder* d, const std::string& name);
int64_t gt_internal_param_offset(gt_decoder* d, const std::string& name);
bool gt_internal_has_param(gt_decoder* d, const std::string& name);
float gt_internal_host_scalar(gt_decoder* d, const std::string& name);
// host copies <- the device fp32 block after gt_decoder_set_params_device (no-op when they are current)
int gt_internal_refresh_host(gt_decoder* d);
const float* gt_internal_freqs(gt_decoder* d);
int64_t gt_internal_numel(gt_decoder* d);
void gt_internal_consts(gt_decoder* d, int* n_spks, float* bmin, float* bmax, float* pe_scale);
int gt_internal_fail(int code, const std::string& msg);
