/*
 * make_output_golden.cpp — fixture generator (test infrastructure only):
 * formats tests/golden/output_items.json the way decode/output.cpp:12-171
 * does, with Qt's own QString::arg / mid / replace and QJsonDocument (conda
 * Qt 5.9.7 in the build container), and writes output_golden.json, which
 * tests/test_host_output.py compares the engine host's formatter against.
 * QString(QByteArray) is spelled fromUtf8(data, size): the reference is a
 * Qt 6 build, where that conversion keeps every byte (Qt 5 stops at NUL).
 * Built and run by make_output_golden.sh; never shipped.
 */
#include <QByteArray>
#include <QDateTime>
#include <QFile>
#include <QJsonArray>
#include <QJsonDocument>
#include <QJsonObject>
#include <QString>
#include <cstdio>

struct Item {
  quint32 AESID;
  quint8 GESID, QNO, REFNO;
  char MODE;
  uchar TAK, BI;
  bool nonacars, downlink, moretocome;
  QByteArray LABEL, PLANEREG;
  QString message;
};

template <typename T>
QString upperHex(T a, int fieldWidth, int base, QChar fillChar) {
  return QString("%1").arg(a, fieldWidth, base, fillChar).toUpper();
}

static QString fmt(int f, const QString &station_id, bool disableReassembly, const Item &item, const QDateTime &time) {
  QByteArray TAKstr;
  TAKstr += item.TAK;
  if (item.TAK == 0x15) TAKstr = ((QString) "!").toLatin1();
  uchar label1 = ' ';
  if (item.LABEL.size() > 1) {
    label1 = item.LABEL[1];
    if ((uchar)item.LABEL[1] == 127) label1 = 'd';
  }
  const QString tak = QString::fromUtf8(TAKstr.constData(), TAKstr.size());
  const QString reg = QString::fromUtf8(item.PLANEREG.constData(), item.PLANEREG.size());
  if (f == 1 || f == 2) {
    QJsonObject root;
    QString message = item.message;
    message.replace('\r', '\n');
    message.replace("\n\n", "\n");
    if (message.right(1) == "\n") message.chop(1);
    if (message.left(1) == "\n") message.remove(0, 1);
    message.replace("\n", "\n\t");
    if (f == 2) {
      QJsonObject app;
      app["name"] = QString("aero-decode");
      app["ver"] = QString("0.0.1");
      root["app"] = QJsonValue(app);
      QJsonObject isu, aes, ges;
      aes["type"] = "Aircraft Earth Station";
      aes["addr"] = upperHex(item.AESID, 6, 16, QChar('0'));
      ges["type"] = "Ground Earth Station";
      ges["addr"] = upperHex(item.GESID, 2, 16, QChar('0'));
      if (!item.nonacars) {
        QJsonObject acars;
        acars["mode"] = (QString)item.MODE;
        acars["ack"] = tak;
        acars["blk_id"] = QString((QChar)item.BI);
        acars["label"] = QString("%1%2").arg(QChar(item.LABEL[0])).arg(QChar(label1));
        acars["reg"] = reg;
        if (!message.isEmpty()) {
          if (item.downlink) {
            acars["msg_num"] = message.mid(0, 3);
            acars["msg_num_seq"] = message.mid(3, 1);
            acars["flight"] = message.mid(4, 6);
            acars["msg_text"] = message.mid(4 + 6);
          } else {
            acars["msg_text"] = message;
          }
        }
        isu["acars"] = QJsonValue(acars);
      }
      isu["refno"] = upperHex(item.REFNO, 2, 16, QChar('0'));
      isu["qno"] = upperHex(item.QNO, 2, 16, QChar('0'));
      isu["src"] = QJsonValue(item.downlink ? aes : ges);
      isu["dst"] = QJsonValue(item.downlink ? ges : aes);
      QJsonObject t;
      QDateTime ts = time.toUTC();
      t["sec"] = ts.toMSecsSinceEpoch() / 1000;
      t["usec"] = (ts.toMSecsSinceEpoch() % 1000) * 1000;
      root["t"] = QJsonValue(t);
      root["isu"] = QJsonValue(isu);
      root["station"] = station_id;
    } else {
      root["TIME"] = time.toMSecsSinceEpoch() / 1000;
      root["TIME_UTC"] = time.toUTC().toString("yyyy-MM-dd hh:mm:ss");
      root["NAME"] = QString("aero-decode");
      root["NONACARS"] = item.nonacars;
      root["AESID"] = upperHex(item.AESID, 6, 16, QChar('0'));
      root["GESID"] = upperHex(item.GESID, 2, 16, QChar('0'));
      root["QNO"] = upperHex(item.QNO, 2, 16, QChar('0'));
      root["REFNO"] = upperHex(item.REFNO, 2, 16, QChar('0'));
      root["REG"] = reg;
      if (!item.nonacars) {
        root["MODE"] = (QString)item.MODE;
        root["TAK"] = tak;
        root["LABEL"] = QString("%1%2").arg(QChar(item.LABEL[0])).arg(QChar(label1));
        root["BI"] = QString((QChar)item.BI);
      }
    }
    return QString::fromUtf8(QJsonDocument(root).toJson(QJsonDocument::Compact));
  }
  QString out;
  QString message = item.message;
  message.replace("\n", "\\n").replace("\r", "\\r").replace("\t", "\\t").replace("\a", "\\a");
  out += QString("%1 AES:%2 GES:%3")
             .arg(time.toUTC().toString("yyyy-MM-ddThh:mm:ssZ"))
             .arg(upperHex(item.AESID, 6, 16, QChar('0')))
             .arg(upperHex(item.GESID, 6, 16, QChar('0')));
  if (!item.nonacars) {
    out += QString(" [%1] ACK=%2 BLK=%3 ").arg(reg, 7).arg(tak, 1).arg(QString((QChar)item.BI));
    if (disableReassembly) out += QString("M=%1 ").arg(item.moretocome ? "1" : "0");
    out += QString("LBL=%1%2 ").arg(QChar(item.LABEL[0])).arg(QChar(label1));
    if (!message.isEmpty()) {
      if (item.downlink)
        out += QString("MSN=%1 FLT=%2 %3").arg(message.mid(0, 4)).arg(message.mid(4, 6)).arg(message.mid(10));
      else
        out += QString("%1").arg(message);
    }
  }
  return out;
}

int main(int argc, char **argv) {
  if (argc != 3) return 2;
  QFile in(argv[1]);
  if (!in.open(QIODevice::ReadOnly)) return 2;
  const QJsonObject doc = QJsonDocument::fromJson(in.readAll()).object();
  const QDateTime time = QDateTime::fromMSecsSinceEpoch((qint64)doc["time_ms"].toDouble(), Qt::UTC);
  const QString station = doc["station"].toString();
  QJsonArray cases;
  for (const QJsonValue &v : doc["items"].toArray()) {
    const QJsonObject o = v.toObject();
    Item it;
    it.AESID = (quint32)o["aesid"].toInt();
    it.GESID = (quint8)o["gesid"].toInt();
    it.QNO = (quint8)o["qno"].toInt();
    it.REFNO = (quint8)o["refno"].toInt();
    it.MODE = (char)o["mode"].toInt();
    it.TAK = (uchar)o["tak"].toInt();
    it.BI = (uchar)o["bi"].toInt();
    it.nonacars = o["nonacars"].toInt() != 0;
    it.downlink = o["downlink"].toInt() != 0;
    it.moretocome = o["moretocome"].toInt() != 0;
    it.LABEL = QByteArray::fromHex(o["label"].toString().toLatin1());
    it.PLANEREG = QByteArray::fromHex(o["reg"].toString().toLatin1());
    const QByteArray m = QByteArray::fromHex(o["msg"].toString().toLatin1());
    it.message.clear();
    for (char c : m) it.message += c;  // ParserISU: message += (char)byte (decode/aerol.cpp:450)
    QJsonObject c;
    c["text"] = fmt(0, station, false, it, time);
    c["text_fragments"] = fmt(0, station, true, it, time);
    c["jaero"] = fmt(1, station, false, it, time);
    c["jsondump"] = fmt(2, station, false, it, time);
    cases.append(c);
  }
  QFile out(argv[2]);
  if (!out.open(QIODevice::WriteOnly)) return 2;
  QJsonObject root;
  root["cases"] = cases;
  root["generator"] = QString("tests/golden/make_output_golden.cpp, Qt ") + QString(qVersion());
  out.write(QJsonDocument(root).toJson(QJsonDocument::Indented));
  return 0;
}
