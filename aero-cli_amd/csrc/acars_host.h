/*
 * acars_host.h — host side of the AeroL P-channel after the GPU has
 * produced a CRC-checked 312-byte information field per frame: SU dispatch
 * (decode/aerol.cpp:1571-1965), ISU/SSU reassembly ISUData
 * (decode/aerol.cpp:158-227), ParserISU (:333-489), ACARSDefragmenter
 * (:229-324), the synchronous empty database lookup
 * (decode/databasetext.cpp:42-61, aerol.cpp:491-524) and the log-on /
 * C-channel-assignment items (aerol.cpp:2099-2143).
 */
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/aero_engine.h"

namespace aero {

struct IsuItem {
  uint32_t aesid = 0;
  uint8_t gesid = 0, qno = 0, seqno = 0, refno = 0, nooct = 0;
  std::string userdata;
  int count = 0;
};

struct AcarsItem {
  IsuItem isu;
  uint8_t mode = 0, tak = 0, bi = 0;
  std::string label, reg, message;
  bool nonacars = false, downlink = false, valid = false, hastext = false, more = false;
};

class PChannelHost {
 public:
  explicit PChannelHost(bool disable_reassembly) : fragments_only_(disable_reassembly) {}
  // one GPU frame record: infofield bytes (len), crc-ok mask, format id
  void frame(const uint8_t *info, int len, uint32_t okmask, int formatid);
  void isu_reset() { isuitems_.clear(); }
  // one decoded burst R/T packet (RTChannelDeleaveFECScram OK_R / OK_T):
  // the R/T branch of AeroL::Decode (decode/aerol.cpp:1253-1460), items
  // marked downlink (parser.downlink = burstmode)
  void rt_packet(bool r_packet, const uint8_t *info, int len, int nsus);
  std::vector<aero_acars_item> items;

 private:
  struct RIsuItem {  // RISUItem (decode/aerol.h:125-135)
    IsuItem isu;
    int seqind = 0, sutype = 0, filled = 0;
  };
  bool risu_update(const uint8_t *d);
  bool isu_update(const uint8_t *d, bool &missing);
  bool parse(const IsuItem &isu);
  bool defragment(AcarsItem &a);
  void emit(const AcarsItem &a, bool fragment);
  void lookup_and_emit(const AcarsItem &a);
  void send_cassign(const uint8_t *info, int k, const std::string &decline);
  void send_logon(const uint8_t *info, int k, const char *text);

  bool fragments_only_;
  bool downlink_ = false;
  std::vector<RIsuItem> risuitems_;
  RIsuItem an_risu_;
  IsuItem risu_last_;
  std::vector<IsuItem> isuitems_;
  IsuItem an_isu_, lastvalid_;
  AcarsItem an_;
  struct Frag {
    AcarsItem item;
    int count;
  };
  std::vector<Frag> frags_;
};

}  // namespace aero
