#include "../../kshim.h"
