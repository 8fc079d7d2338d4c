#pragma once
#include <stdio.h>
