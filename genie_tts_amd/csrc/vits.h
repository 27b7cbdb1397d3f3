// VITS (SoVITS decoder + HiFi-GAN) device weights and workspace.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsv {
struct VitsWeights {
    bool ready = false;
};
struct VitsWorkspace {
    size_t cap = 0;
};
struct PromptEncWeights {
    bool ready = false;
};
}  // namespace gsv
