// TEST-ONLY stand-in (see ../core/core.hpp): cv::KeyPoint lives there.
#pragma once
#include "../core/core.hpp"
