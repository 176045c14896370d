/*
 * ref_wt901_harness.c -- driver around the REFERENCE's own WT901 SDK
 * (lib/wt901c/wit_c_sdk.c, compiled unmodified from /root/reference by
 * oracle/Makefile into oracle/_ref/libwit_ref.so).
 *
 * TEST INFRASTRUCTURE ONLY.  This is not a stand-in for anything the SDK needs:
 * wit_c_sdk.c includes only <stdint.h>, <stdio.h>, <string.h> and its own REG.h.
 * The harness only registers callbacks the way IMU_IF_WT901C::init does
 * (src/Imu/imu_if_wt901c.cpp:63-69) and records what the SDK reports, so the
 * golden fixtures in tests/golden/ can pin the oracle's parser restatement.
 */
#include <stdint.h>
#include <string.h>

#include "wit_c_sdk.h"

#define LOGMAX 4096
static uint16_t g_cb_reg[LOGMAX], g_cb_num[LOGMAX];
static uint32_t g_ncb;

static void harness_cb(uint32_t reg, uint32_t num) {
  if (g_ncb < LOGMAX) {
    g_cb_reg[g_ncb] = (uint16_t)reg;
    g_cb_num[g_ncb] = (uint16_t)num;
    g_ncb++;
  }
}

static void harness_serial_write(uint8_t *p, uint32_t n) {
  (void)p;
  (void)n;
}

/* Fresh parser: WitInit resets the byte count; sReg is zeroed (static storage at boot). */
int ref_wt901_begin(uint32_t read_reg_index) {
  WitInit(WIT_PROTOCOL_NORMAL, 0x50);
  WitSerialWriteRegister(harness_serial_write);
  WitRegisterCallBack(harness_cb);
  memset(sReg, 0, sizeof(int16_t) * REGSIZE);
  g_ncb = 0;
  /* WitReadReg records the register index later 0x5F (REGVALUE) frames write to */
  return WitReadReg(read_reg_index, 1);
}

void ref_wt901_feed(const uint8_t *bytes, uint32_t len) {
  for (uint32_t i = 0; i < len; i++) WitSerialDataIn(bytes[i]);
}

void ref_wt901_regs(int16_t *out) { memcpy(out, sReg, sizeof(int16_t) * REGSIZE); }

/* returns the number of callbacks since the last call and clears the log */
uint32_t ref_wt901_take_cb(uint16_t *reg, uint16_t *num, uint32_t max) {
  uint32_t n = g_ncb < max ? g_ncb : max;
  memcpy(reg, g_cb_reg, n * sizeof(uint16_t));
  memcpy(num, g_cb_num, n * sizeof(uint16_t));
  g_ncb = 0;
  return n;
}
