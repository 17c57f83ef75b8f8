// placeholder
#include "skv_launch.hpp"
