// test stub: the reference package's Channel<T> interface (LeGO-LOAM/include/lego_loam/channel.h:11-56:
// one writer / one reader, optionally blocking send), declarations only
#pragma once
template <class T>
class Channel {
 public:
  Channel(bool blocking_send);
  void send(T&& item);
  void send(const T& item);
  void receive(T& item);
};
