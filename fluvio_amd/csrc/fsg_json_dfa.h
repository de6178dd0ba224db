// fsg_json_dfa.h — the token DFA of the lean filter_json path (fsg_kernels.hip
// lean_json_stage).  Input: the tokens of one record value — every quote,
// every special byte (< 0x20, '\\', >= 0x80) and every non-space byte outside
// strings — each with an "adjacent to the previous token" bit.  Opening quotes
// carry the class of their string.  The DFA accepts exactly the flat objects
// whose serde_json::from_slice::<StructuredLog> outcome is certain
// (smartmodule/examples/filter_json/src/lib.rs:54-70; de.rs deserialize_struct,
// MapAccess, deserialize_enum, deserialize_str, ignore_value /
// ignore_integer / ignore_decimal / ignore_exponent):
//   { "key": value (, "key": value)* }   keys and strings without escapes,
//   level: a LogLevel variant string, message: a string, other values: a
//   string, a JSON number or true / false / null.
// Everything else ends in JS_FAIL and the record goes to the exact
// restatement (fsg_json_dev.h).  Each field at most once is checked beside
// the table (a duplicate field is a serde error).
#pragma once
#include <cstdint>

namespace fsg {

enum JsonTokCls : uint8_t {
  JC_LBRACE, JC_RBRACE, JC_COLON, JC_COMMA,
  JC_Q_OTHER, JC_Q_LEVEL, JC_Q_MSG, JC_Q_DEBUG, JC_Q_INFO, JC_Q_WARN, JC_Q_ERROR, JC_Q_CLOSE,
  JC_D0, JC_D19, JC_MINUS, JC_DOT, JC_e, JC_E, JC_PLUS,
  JC_t, JC_r, JC_u, JC_f, JC_a, JC_l, JC_s, JC_n,
  JC_OTHER,
  JC_COUNT,
  JC_Q_FIELD = JC_COUNT  // projection: a string equal to the field name (taken as JC_Q_OTHER by the table)
};
enum JsonTokState : uint8_t {
  JS_OBJ, JS_KEY_OR_END, JS_KEY, JS_INKEY_LV, JS_INKEY_MSG, JS_INKEY_OTHER,
  JS_COLON_LV, JS_COLON_MSG, JS_COLON_OTHER, JS_VAL_LV, JS_VAL_MSG, JS_VAL_OTHER,
  JS_INV_D, JS_INV_I, JS_INV_W, JS_INV_E, JS_INSTR, JS_AFTER, JS_END,
  JS_N_MINUS, JS_N_ZERO, JS_N_INT, JS_N_DOT, JS_N_FRAC, JS_N_E, JS_N_ESIGN, JS_N_EXP,
  JS_T1, JS_T2, JS_T3, JS_F1, JS_F2, JS_F3, JS_F4, JS_N1, JS_N2, JS_N3,
  JS_FAIL,
  JS_COUNT
};
constexpr int kJsonStates = JS_COUNT;
constexpr int kJsonCls2 = 2 * JC_COUNT;  // (class, adjacent)

struct JsonDfaTables {
  uint8_t t[kJsonStates * kJsonCls2];
  uint8_t bcls[256];
  constexpr JsonDfaTables() : t(), bcls() {
    for (int i = 0; i < kJsonStates * kJsonCls2; i++) t[i] = JS_FAIL;
    for (int b = 0; b < 256; b++) bcls[b] = JC_OTHER;
    bcls['{'] = JC_LBRACE;
    bcls['}'] = JC_RBRACE;
    bcls[':'] = JC_COLON;
    bcls[','] = JC_COMMA;
    bcls['"'] = JC_Q_OTHER;  // refined per token (opening class / closing)
    bcls['0'] = JC_D0;
    for (int b = '1'; b <= '9'; b++) bcls[b] = JC_D19;
    bcls['-'] = JC_MINUS;
    bcls['.'] = JC_DOT;
    bcls['e'] = JC_e;
    bcls['E'] = JC_E;
    bcls['+'] = JC_PLUS;
    bcls['t'] = JC_t;
    bcls['r'] = JC_r;
    bcls['u'] = JC_u;
    bcls['f'] = JC_f;
    bcls['a'] = JC_a;
    bcls['l'] = JC_l;
    bcls['s'] = JC_s;
    bcls['n'] = JC_n;
    // structure
    both(JS_OBJ, JC_LBRACE, JS_KEY_OR_END);
    for (int s : {JS_KEY_OR_END, JS_KEY}) {
      both(s, JC_Q_LEVEL, JS_INKEY_LV);
      both(s, JC_Q_MSG, JS_INKEY_MSG);
      for (int c : {JC_Q_OTHER, JC_Q_DEBUG, JC_Q_INFO, JC_Q_WARN, JC_Q_ERROR}) both(s, c, JS_INKEY_OTHER);
    }
    both(JS_INKEY_LV, JC_Q_CLOSE, JS_COLON_LV);
    both(JS_INKEY_MSG, JC_Q_CLOSE, JS_COLON_MSG);
    both(JS_INKEY_OTHER, JC_Q_CLOSE, JS_COLON_OTHER);
    both(JS_COLON_LV, JC_COLON, JS_VAL_LV);
    both(JS_COLON_MSG, JC_COLON, JS_VAL_MSG);
    both(JS_COLON_OTHER, JC_COLON, JS_VAL_OTHER);
    both(JS_VAL_LV, JC_Q_DEBUG, JS_INV_D);
    both(JS_VAL_LV, JC_Q_INFO, JS_INV_I);
    both(JS_VAL_LV, JC_Q_WARN, JS_INV_W);
    both(JS_VAL_LV, JC_Q_ERROR, JS_INV_E);
    for (int c = JC_Q_OTHER; c <= JC_Q_ERROR; c++) {
      both(JS_VAL_MSG, c, JS_INSTR);
      both(JS_VAL_OTHER, c, JS_INSTR);
    }
    both(JS_VAL_OTHER, JC_D0, JS_N_ZERO);
    both(JS_VAL_OTHER, JC_D19, JS_N_INT);
    both(JS_VAL_OTHER, JC_MINUS, JS_N_MINUS);
    both(JS_VAL_OTHER, JC_t, JS_T1);
    both(JS_VAL_OTHER, JC_f, JS_F1);
    both(JS_VAL_OTHER, JC_n, JS_N1);
    for (int s : {JS_INV_D, JS_INV_I, JS_INV_W, JS_INV_E, JS_INSTR}) both(s, JC_Q_CLOSE, JS_AFTER);
    after(JS_AFTER);
    // numbers: continuations must be adjacent; a final state ends like AFTER
    for (int s : {JS_N_ZERO, JS_N_INT, JS_N_FRAC, JS_N_EXP}) after(s);
    adj(JS_N_MINUS, JC_D0, JS_N_ZERO);
    adj(JS_N_MINUS, JC_D19, JS_N_INT);
    adj(JS_N_ZERO, JC_DOT, JS_N_DOT);
    adj(JS_N_ZERO, JC_e, JS_N_E);
    adj(JS_N_ZERO, JC_E, JS_N_E);
    for (int c : {JC_D0, JC_D19}) {
      adj(JS_N_INT, c, JS_N_INT);
      adj(JS_N_DOT, c, JS_N_FRAC);
      adj(JS_N_FRAC, c, JS_N_FRAC);
      adj(JS_N_E, c, JS_N_EXP);
      adj(JS_N_ESIGN, c, JS_N_EXP);
      adj(JS_N_EXP, c, JS_N_EXP);
    }
    for (int c : {JC_e, JC_E}) {
      adj(JS_N_INT, c, JS_N_E);
      adj(JS_N_FRAC, c, JS_N_E);
    }
    adj(JS_N_INT, JC_DOT, JS_N_DOT);
    adj(JS_N_E, JC_PLUS, JS_N_ESIGN);
    adj(JS_N_E, JC_MINUS, JS_N_ESIGN);
    // literals true / false / null, letter by adjacent letter
    adj(JS_T1, JC_r, JS_T2);
    adj(JS_T2, JC_u, JS_T3);
    adj(JS_T3, JC_e, JS_AFTER);
    adj(JS_F1, JC_a, JS_F2);
    adj(JS_F2, JC_l, JS_F3);
    adj(JS_F3, JC_s, JS_F4);
    adj(JS_F4, JC_e, JS_AFTER);
    adj(JS_N1, JC_u, JS_N2);
    adj(JS_N2, JC_l, JS_N3);
    adj(JS_N3, JC_l, JS_AFTER);
  }
  constexpr void set(int s, int c, int a, int to) { t[s * kJsonCls2 + c * 2 + a] = (uint8_t)to; }
  constexpr void both(int s, int c, int to) {
    set(s, c, 0, to);
    set(s, c, 1, to);
  }
  constexpr void adj(int s, int c, int to) { set(s, c, 1, to); }
  // after a complete value: ',' -> next key, '}' -> end (adjacent or not)
  constexpr void after(int s) {
    both(s, JC_COMMA, JS_KEY);
    both(s, JC_RBRACE, JS_END);
  }
};

constexpr JsonDfaTables kJsonDfa{};

}  // namespace fsg
