/*
 * The connectors' packet loops with the SRTP step kept in flight on the GPU.
 *
 * The reference runs SRTP synchronously, one packet at a time, inside each
 * connector thread: the send thread of RTPConnectorOutputStream's queue takes a
 * buffer, packetizes it -- TransformUDPOutputStream.packetize runs the whole
 * transformer chain, SRTP last -- and writes the packets
 * (RTPConnectorOutputStream.java:775-835, packetize :268-300); the receive
 * thread receives one datagram, and TransformInputStream.createRawPacket runs
 * the reverse chain, SRTP first, before transferData
 * (RTPConnectorInputStream.java:425-452,780-806).  Through GpuTransformerBase's
 * per-packet call that is one GPU round trip per packet per thread.
 *
 * Send and Receive below are those two loops with the SRTP step taken out of
 * the chain and put through a GpuPacketQueue: a thread submits every packet it
 * has, keeps going while they are on the GPU, and sends (hands on) each result
 * in submission order as it is reaped -- so the order on the wire and to the
 * jitter buffer is the reference's, and so are the bytes (the engine is the
 * reference's SRTP, bit for bit).  A packet the reference drops (replay, auth)
 * is not sent / not handed on, as there; one on which SRTPCryptoContext throws
 * is counted and logged as SinglePacketTransformer does and dropped.
 *
 * The integration (INTEGRATION.md, "Connector loops"): RTPConnectorOutputStream
 * .Queue.runInSendThread delegates to Send.run when its stream's SRTP
 * transformer is a GpuTransformerBase, with its queue poll, its packetize over
 * the chain without the SRTP engine, its pool, its pacing + write(RawPacket[])
 * as the callbacks; RTPConnectorInputStream.runInReceiveThread likewise to
 * Receive.run with its receive (a short socket timeout while results are
 * outstanding), accept, createRawPacket without the reverse chain, the reverse
 * chain after SRTP, and transferData.
 *
 * Not compiled in this repository (no JDK).  The loops' logic -- when to poll,
 * submit, reap with and without waiting -- is driven against the oracle in C
 * through the stand-in JVM (tests/jni_stub/fakejvm.c fj_send_loop /
 * fj_receive_loop, tests/test_jni_shim.py).
 */
package org.jitsi.impl.neomedia.transform.srtp.mi355x;

import java.io.*;
import java.net.*;

import org.jitsi.impl.neomedia.*;

public final class GpuConnectorLoops
{
    /** Packets a connector thread keeps in flight. */
    public static final int IN_FLIGHT = 256;

    /** How long an idle thread waits for new input while none is in flight (the reference's poll, :790). */
    static final long IDLE_POLL_MS = 500;

    private GpuConnectorLoops()
    {
    }

    /** The send thread's side of RTPConnectorOutputStream.Queue. */
    public interface SendSide
    {
        boolean closed();

        /** Queue.queue.poll(timeout) (:787-795); null when nothing came. */
        Object poll(long timeoutMs)
            throws InterruptedException;

        /**
         * packetize(buffer.buf, 0, buffer.len, buffer.context) with the
         * transformer chain up to, not including, the SRTP engine; then the
         * buffer goes back to Queue.pool (:806-811).
         */
        RawPacket[] packetize(Object buffer);

        /** The pacing of :813-827 and RTPConnectorOutputStream.write(RawPacket[]) (:829). */
        void send(RawPacket pkt);
    }

    public static final class Send
    {
        private final SendSide side;

        private final GpuTransformerBase srtp;

        private final GpuPacketQueue q = new GpuPacketQueue(IN_FLIGHT);

        private final GpuPacketQueue.Sink sink;

        public Send(SendSide side, GpuTransformerBase srtp)
        {
            this.side = side;
            this.srtp = srtp;
            this.sink = pkt -> {
                if (pkt != null)
                    side.send(pkt);
            };
        }

        public void run()
        {
            try
            {
                while (!side.closed())
                {
                    Object buffer;
                    try
                    {
                        // with packets on the GPU, do not sleep on an empty
                        // queue: their results are due
                        buffer = side.poll(q.outstanding() > 0 ? 0 : IDLE_POLL_MS);
                    }
                    catch (InterruptedException iex)
                    {
                        continue;
                    }
                    if (buffer == null)
                    {
                        if (q.outstanding() > 0)
                            q.reap(sink, true);
                        continue;
                    }
                    for (RawPacket pkt : side.packetize(buffer))
                        if (pkt != null)
                            q.transform(srtp, pkt, false, sink);
                    q.reap(sink, false); // hand on whatever is done, without waiting
                }
                q.drain(sink);
            }
            finally
            {
                q.close();
            }
        }
    }

    /** The receive thread's side of RTPConnectorInputStream. */
    public interface ReceiveSide
    {
        boolean closed();

        /**
         * receive(p) (:784) with a socket timeout of timeoutMs (0: block):
         * false when it timed out.
         */
        boolean receive(DatagramPacket p, int timeoutMs)
            throws IOException;

        /** accept(p) (:793). */
        boolean accept(DatagramPacket p);

        /** RTPConnectorInputStream.createRawPacket (:425-452): the copy, no transformer. */
        RawPacket[] createRawPacket(DatagramPacket p);

        /**
         * The reverse transformer chain after the SRTP engine, the datagram
         * listeners and transferData (:795-797).
         */
        void handOn(RawPacket pkt);
    }

    public static final class Receive
    {
        private final ReceiveSide side;

        private final GpuTransformerBase srtp;

        private final GpuPacketQueue q = new GpuPacketQueue(IN_FLIGHT);

        private final GpuPacketQueue.Sink sink;

        public Receive(ReceiveSide side, GpuTransformerBase srtp)
        {
            this.side = side;
            this.srtp = srtp;
            this.sink = pkt -> {
                if (pkt != null)
                    side.handOn(pkt);
            };
        }

        /** Returns normally on close; an IOException ends the loop as there (ioError, :786-789). */
        public void run(DatagramPacket p)
            throws IOException
        {
            try
            {
                while (!side.closed())
                {
                    // results outstanding: wait for the socket only briefly
                    if (!side.receive(p, q.outstanding() > 0 ? 1 : 0))
                    {
                        q.reap(sink, true);
                        continue;
                    }
                    if (side.accept(p))
                        for (RawPacket pkt : side.createRawPacket(p))
                            if (pkt != null)
                                q.transform(srtp, pkt, true, sink);
                    q.reap(sink, false);
                }
                q.drain(sink);
            }
            finally
            {
                q.close();
            }
        }
    }
}
