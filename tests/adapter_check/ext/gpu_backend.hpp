// Test infrastructure: the adapter includes "gpu_backend.hpp"; this forwards to the restated interface.
#pragma once
#include "gpu_backend_decl.hpp"
