#include "../kshim.h"
