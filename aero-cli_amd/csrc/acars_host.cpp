/*
 * acars_host.cpp — see acars_host.h.  Runs on the host per decoded frame
 * (2 per second per channel); its outputs are part of the parity contract.
 */
#include "acars_host.h"

#include <algorithm>
#include <cstdio>
#include <cstring>

namespace aero {

namespace {
uint32_t aes_of(const uint8_t *info, int k) {  // infofield[k*12-1+2..4] (aerol.cpp:2101-2103)
  return (uint32_t)info[k * 12 - 1 + 2] << 16 | (uint32_t)info[k * 12 - 1 + 3] << 8 | info[k * 12 - 1 + 4];
}
}  // namespace

void PChannelHost::emit(const AcarsItem &a, bool fragment) {
  aero_acars_item o;
  memset(&o, 0, sizeof o);
  o.aesid = a.isu.aesid;
  o.gesid = a.isu.gesid;
  o.qno = a.isu.qno;
  o.refno = a.isu.refno;
  o.seqno = a.isu.seqno;
  o.mode = a.mode;
  o.tak = a.tak;
  o.bi = a.bi;
  o.nonacars = a.nonacars;
  o.downlink = a.downlink;
  o.valid = a.valid;
  o.hastext = a.hastext;
  o.moretocome = a.more;
  o.fragment = fragment ? 1 : 0;
  o.label_len = (uint8_t)std::min<size_t>(a.label.size(), sizeof o.label);
  memcpy(o.label, a.label.data(), o.label_len);
  o.reg_len = (uint8_t)std::min<size_t>(a.reg.size(), sizeof o.reg);
  memcpy(o.reg, a.reg.data(), o.reg_len);
  o.msg_len = (uint32_t)std::min<size_t>(a.message.size(), sizeof o.msg);
  memcpy(o.msg, a.message.data(), o.msg_len);
  items.push_back(o);
}

// ISUData::update (aerol.cpp:158-227); `an_isu_` keeps the reference's member
// reuse: an SSU inherits AESID/GESID/NOOCT of the last 0x71 seen.
bool PChannelHost::isu_update(const uint8_t *d, bool &missing) {
  missing = false;
  const uint8_t message = d[0];
  if (message == 0x71) {
    for (size_t i = 0; i < isuitems_.size(); i++) {  // deleteoldisuitems
      if (++isuitems_[i].count > 10) {
        isuitems_.erase(isuitems_.begin() + i);
        i--;
      }
    }
    an_isu_.aesid = (uint32_t)d[1] << 16 | (uint32_t)d[2] << 8 | d[3];
    an_isu_.gesid = d[4];
    an_isu_.qno = (d[5] >> 4) & 0x0F;
    an_isu_.refno = d[5] & 0x0F;
    an_isu_.seqno = d[6] & 0x3F;
    an_isu_.nooct = (d[7] >> 4) & 0x0F;
    an_isu_.count = 0;
    an_isu_.userdata.assign(reinterpret_cast<const char *>(d + 8), 2);
    int idx = -1;
    if (an_isu_.nooct <= 8)
      for (size_t i = 0; i < isuitems_.size(); i++)
        if (an_isu_.aesid == isuitems_[i].aesid && an_isu_.gesid == isuitems_[i].gesid &&
            an_isu_.qno == isuitems_[i].qno && an_isu_.refno == isuitems_[i].refno) {
          idx = (int)i;
          break;
        }
    if (idx < 0)
      isuitems_.push_back(an_isu_);
    else
      isuitems_[idx] = an_isu_;
    return false;
  }
  if ((message & 0xC0) != 0xC0) return false;
  an_isu_.seqno = message & 0x3F;
  an_isu_.qno = (d[1] >> 4) & 0x0F;
  an_isu_.refno = d[1] & 0x0F;
  int idx = -1;
  if (an_isu_.nooct <= 8)
    for (size_t i = 0; i < isuitems_.size(); i++)
      if (an_isu_.aesid == isuitems_[i].aesid && an_isu_.gesid == isuitems_[i].gesid &&
          (uint8_t)(an_isu_.seqno + 1) == isuitems_[i].seqno && an_isu_.qno == isuitems_[i].qno &&
          an_isu_.refno == isuitems_[i].refno) {
        idx = (int)i;
        break;
      }
  if (idx < 0) {
    missing = true;
    return false;
  }
  IsuItem &it = isuitems_[idx];
  it.seqno--;
  if (it.seqno == 0) {
    for (int i = 2; i <= it.nooct + 1; i++) it.userdata += (char)d[i];
    lastvalid_ = it;
    return true;
  }
  for (int i = 2; i <= 9; i++) it.userdata += (char)d[i];
  return false;
}

// ACARSDefragmenter::defragment (aerol.cpp:281-324)
bool PChannelHost::defragment(AcarsItem &a) {
  for (size_t i = 0; i < frags_.size(); i++) {
    if (++frags_[i].count > 30) {
      frags_.erase(frags_.begin() + i);
      i--;
    }
  }
  int idx = -1;
  for (size_t i = 0; i < frags_.size(); i++) {
    const AcarsItem &p = frags_[i].item;
    if (a.reg == p.reg && a.label == p.label && a.mode == p.mode && a.isu.aesid == p.isu.aesid &&
        a.isu.gesid == p.isu.gesid && p.more) {
      if (a.tak != p.tak) continue;
      const uint8_t expnewbi = (uint8_t)((((p.bi + 1) - 'A') % 26) + 'A');
      if (expnewbi == a.bi) {
        idx = (int)i;
        break;
      }
    }
  }
  if (idx < 0) {
    if (!a.more) return true;
    frags_.push_back({a, 0});
    return false;
  }
  Frag &o = frags_[idx];
  o.count = 0;
  o.item.bi = a.bi;
  o.item.message += a.message;
  o.item.more = a.more;
  if (a.more) return false;
  a = o.item;
  frags_.erase(frags_.begin() + idx);
  return true;
}

// DataBaseTextUser::request -> acarslookupresult with an empty result
void PChannelHost::lookup_and_emit(const AcarsItem &in) {
  AcarsItem p = in;
  size_t i = 0;
  while (i < p.reg.size() && p.reg[i] == '.') i++;
  p.reg = p.reg.substr(i);
  if (!fragments_only_) emit(p, false);
}

// ParserISU::parse (aerol.cpp:333-489); downlink is false on the P channel, true on R/T
bool PChannelHost::parse(const IsuItem &isu) {
  if (isu.aesid == 0) return false;
  const std::string &ud = isu.userdata;
  std::vector<uint8_t> par(ud.size());
  std::string textish;
  for (size_t i = 0; i < ud.size(); i++) {
    const int b = (uint8_t)ud[i];
    par[i] = __builtin_popcount(b) & 1;
    textish += (char)(b & 0x7F);
  }
  const bool isacars = ud.size() > 16 && (uint8_t)ud[0] == 0xFF && (uint8_t)ud[1] == 0xFF &&
                       ((uint8_t)ud[15] == 0x83 || (uint8_t)ud[15] == 0x02);
  if (isacars) {
    an_ = AcarsItem();
    an_.downlink = downlink_;
    an_.isu = isu;
    an_.mode = (uint8_t)ud[3] & 0x7F;
    an_.tak = (uint8_t)textish[11];
    an_.label += textish[12];
    an_.label += textish[13];
    an_.bi = (uint8_t)textish[14];
    if ((uint8_t)ud[15] == 0x02) an_.hastext = true;
    if ((uint8_t)ud[ud.size() - 1 - 3] == 0x97) an_.more = true;
    for (int k = 4; k < 4 + 7; k++) {
      if (!par[k]) return false;
      an_.reg += (char)((uint8_t)ud[k] & 0x7F);
    }
    if (an_.hastext) {
      for (int k = 16; k < (int)ud.size() - 1 - 3; k++) {
        const uint8_t b = (uint8_t)ud[k] & 0x7F;
        if (!par[k]) return false;
        if (b == 0x7F)
          an_.message += "<DEL>";
        else
          an_.message += (char)b;
      }
    }
    an_.valid = true;
    if (fragments_only_) emit(an_, true);
    if (defragment(an_)) lookup_and_emit(an_);
    return true;
  }
  an_ = AcarsItem();
  an_.downlink = downlink_;
  an_.isu = isu;
  an_.nonacars = true;
  static const char *H = "0123456789ABCDEF";
  for (unsigned char b : ud) {
    an_.message += H[b >> 4];
    an_.message += H[b & 15];
  }
  an_.valid = true;
  lookup_and_emit(an_);
  return true;
}

void PChannelHost::send_cassign(const uint8_t *info, int k, const std::string &decline) {
  AcarsItem item;
  item.isu.aesid = aes_of(info, k);
  item.isu.gesid = info[k * 12 - 1 + 5];
  item.hastext = item.downlink = item.nonacars = item.valid = true;
  const int b7 = info[k * 12 - 1 + 7], b8 = info[k * 12 - 1 + 8];
  const int b9 = info[k * 12 - 1 + 9], b10 = info[k * 12 - 1 + 10];
  const int ch1 = ((((b7 & 0x7F) << 8) & 0xFF00) | (b8 & 0x00FF));
  const int ch2 = ((((b9 & 0x7F) << 8) & 0xFF00) | (b10 & 0x00FF));
  char rx[48], tx[48];
  snprintf(rx, sizeof rx, "%.4f", (((double)ch1) * 0.0025) + 1510.0);
  snprintf(tx, sizeof tx, "%.4f", (((double)ch2) * 0.0025) + 1611.5);
  item.message = std::string("Receive Freq: ") + rx + ((b7 & 0x80) ? " Spot Beam " : " Global Beam ") +
                 "Transmit " + tx + "\r\n" + decline;
  if (!fragments_only_) emit(item, false);
}

void PChannelHost::send_logon(const uint8_t *info, int k, const char *text) {
  AcarsItem item;
  item.isu.aesid = aes_of(info, k);
  item.isu.gesid = info[k * 12 - 1 + 5];
  item.hastext = item.downlink = item.nonacars = item.valid = true;
  item.message = text;
  if (!fragments_only_) emit(item, false);
}

// SU k's line of the reference's per-frame `decline` text (aerol.cpp:1522-1536):
// only C-channel-assignment items carry it, so it is built on demand.
static std::string decline_prefix(const uint8_t *su, int k, int formatid) {
  static const char H[] = "0123456789ABCDEF";
  std::string d;
  if (k == 0 && formatid != 1) d += "format ID error\n";
  d += (char)(k + '0');
  for (int j = 0; j < 10; j++) {
    const char b[6] = {' ', '0', 'x', H[su[j] >> 4], H[su[j] & 15], 0};
    d += b;
  }
  d += ' ';
  return d;
}

// frame-done SU loop (aerol.cpp:1522-1990): only the branches that emit items
void PChannelHost::frame(const uint8_t *info, int len, uint32_t okmask, int formatid) {
  for (int k = 0; k < len / 12; k++) {
    if (!(okmask & (1u << k))) continue;
    const uint8_t *su = info + 12 * k;
    const uint8_t m = su[0];
    bool missing;
    const char *what = nullptr;
    switch (m) {
      case 0x11:
        send_logon(info, k, "Log on confirm");
        break;
      case 0x31: what = "C_channel_assignment_distress"; break;
      case 0x32: what = "C_channel_assignment_flight_safety"; break;
      case 0x33: what = "C_channel_assignment_other_safety"; break;
      case 0x34: what = "C_channel_assignment_non_safety"; break;
      case 0x21: what = "Call_announcement"; break;
      case 0x71:
        isu_update(su, missing);
        break;
      default:
        if ((m & 0xC0) == 0xC0 && isu_update(su, missing)) parse(lastvalid_);
        break;
    }
    if (what) send_cassign(info, k, decline_prefix(su, k, formatid) + what);
  }
}

// RISUData::update (decode/aerol.cpp:32-119) on the first 17 bytes of an R packet
bool PChannelHost::risu_update(const uint8_t *d) {
  for (size_t i = 0; i < risuitems_.size(); i++) {  // deleteoldisuitems
    risuitems_[i].isu.count++;
    if (risuitems_[i].isu.count > 10) {
      risuitems_.erase(risuitems_.begin() + i);
      i--;
    }
  }
  const int byte1 = d[0], byte2 = d[1], byte3 = d[2], byte4 = d[3], byte5 = d[4], byte6 = d[5];
  an_risu_ = RIsuItem();
  an_risu_.seqind = ((byte1 & 0xF0) >> 4);
  an_risu_.sutype = byte1 & 0x0F;
  an_risu_.isu.qno = (uint8_t)((byte2 & 0xF0) >> 4);
  an_risu_.isu.refno = (uint8_t)(byte2 & 0x07);
  an_risu_.isu.aesid = (uint32_t)(byte3 << 16 | byte4 << 8 | byte5);
  an_risu_.isu.gesid = (uint8_t)byte6;
  int idx = -1;
  if (an_risu_.sutype >= 1 && an_risu_.sutype <= 11)
    for (size_t i = 0; i < risuitems_.size(); i++)
      if (an_risu_.isu.gesid == risuitems_[i].isu.gesid && an_risu_.isu.aesid == risuitems_[i].isu.aesid &&
          an_risu_.isu.qno == risuitems_[i].isu.qno && an_risu_.isu.refno == risuitems_[i].isu.refno) {
        idx = (int)i;
        break;
      }
  if (idx < 0) {
    risuitems_.push_back(an_risu_);
    idx = (int)risuitems_.size() - 1;
  }
  RIsuItem *p = &risuitems_[idx];
  p->isu.count = 0;
  int su_total = 0, su_index = 0;
  switch (an_risu_.seqind) {
    case 1: su_total = 1; su_index = 0; break;
    case 2: su_total = 2; su_index = 0; break;
    case 3: su_total = 2; su_index = 1; break;
    case 4: su_total = 3; su_index = 0; break;
    case 5: su_total = 3; su_index = 1; break;
    case 6: su_total = 3; su_index = 2; break;
    default: break;
  }
  int bytes_in_su = 0;
  if ((an_risu_.sutype >= 1) && (an_risu_.sutype <= 11)) bytes_in_su = an_risu_.sutype;
  const bool signaling = an_risu_.sutype == 15;
  const int thisnum = 11 * su_total - 11 + bytes_in_su;
  if (thisnum > 0) {
    if (p->isu.userdata.size() == 0) p->isu.userdata.resize(thisnum);
    if (thisnum < (int)p->isu.userdata.size()) p->isu.userdata.resize(thisnum);
  }
  if (!signaling) {
    for (int i = 0 - 1 + 7; i < bytes_in_su - 1 + 7; i++) {
      // QByteArray's operator[] grows the array on an out-of-range write
      const size_t at = (size_t)(i + 11 * su_index + 1 - 7);
      if (at >= p->isu.userdata.size()) p->isu.userdata.resize(at + 1, '\0');
      p->isu.userdata[at] = (char)d[i];
    }
    p->filled |= (1 << su_index);
  } else {
    p->isu.userdata.clear();
  }
  if ((signaling) || ((p->filled == 7) && (su_total == 3)) || ((p->filled == 3) && (su_total == 2)) ||
      ((p->filled == 1) && (su_total == 1))) {
    risu_last_ = p->isu;
    risuitems_.erase(risuitems_.begin() + idx);
    return true;
  }
  return false;
}

void PChannelHost::rt_packet(bool r_packet, const uint8_t *info, int len, int nsus) {
  downlink_ = true;
  if (r_packet) {  // User_data_ISU_SSU_R_channel (aerol.cpp:1256-1290)
    if (len >= 17 && (info[1] & 0x08) == 0x08 && risu_update(info)) parse(risu_last_);
    return;
  }
  for (int k = 0; k < nsus; k++) {  // T channel SUs (aerol.cpp:1300-1460)
    if (6 + k * 12 + 10 > len) break;
    const uint8_t *su = info + 6 + k * 12;
    int message = su[0];
    if ((message & 0xC0) == 0xC0) message = -1;
    bool missing;
    if (message == 0x71) {
      isu_update(su, missing);
    } else if (message == -1) {
      if (isu_update(su, missing)) parse(lastvalid_);
    }
  }
}

}  // namespace aero
