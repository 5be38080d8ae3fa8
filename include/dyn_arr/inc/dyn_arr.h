/* compatibility path: reference layout dyn_arr/inc/dyn_arr.h */
#include "../../dyn_arr.h"
