/*
 * The asynchronous per-packet transform for a thread that has many packets at
 * hand: a connector's send thread draining its queue
 * (RTPConnectorOutputStream.Queue.runInSendThread, RTPConnectorOutputStream.java
 * :652-830), or a receive loop handing on each datagram
 * (RTPConnectorInputStream.java:425-452,780-806).  The reference transforms
 * those packets one call at a time (SinglePacketTransformer.transform(RawPacket),
 * :113,169); through GpuTransformerBase's per-packet call a thread has one packet
 * in flight.  Here it submits every packet it has, reaps the results in
 * submission order and sends (or hands on) each, so one thread keeps up to
 * maxInFlight packets in the GPU's bundles.
 *
 * Not compiled in this repository (no JDK); the native half
 * (queueCreate/Submit/Reap/Destroy in src/native/srtp_mi355x/SrtpMi355x.c over
 * srtp_queue_* and srtp_rawpacket_submit/_complete) is, and is tested through a
 * stand-in JVM (tests/test_jni_shim.py).  See INTEGRATION.md.
 */
package org.jitsi.impl.neomedia.transform.srtp.mi355x;

import org.jitsi.impl.neomedia.*;
import org.jitsi.util.*;

public final class GpuPacketQueue
{
    /** Receives each reaped packet, or null where the reference drops it. */
    public interface Sink
    {
        void accept(RawPacket pkt);
    }

    /** SinglePacketTransformer.EXCEPTIONS_TO_LOG (:42) */
    private static final int EXCEPTIONS_TO_LOG = 1000;

    private static final Logger logger = Logger.getLogger(GpuPacketQueue.class);

    private final long q;

    /** Packets in flight, by submission number (the native cookie). */
    private final RawPacket[] ring;

    private final int[] status;

    private long submitted, reaped;

    private long exceptions;

    /**
     * A queue of one thread (submit and reap are not thread-safe) on the
     * process's aggregator.
     */
    public GpuPacketQueue(int maxInFlight)
    {
        if (maxInFlight < 1)
            throw new IllegalArgumentException("maxInFlight");
        ring = new RawPacket[maxInFlight];
        status = new int[Math.min(maxInFlight, 1024)];
        q = SrtpMi355x.queueCreate(SrtpMi355x.aggregator(), maxInFlight);
        if (q == 0)
            throw new IllegalStateException("srtp_mi355x: no queue");
    }

    /**
     * Starts transformer t's transform (reverse = false) or reverseTransform
     * (reverse = true) of pkt.  The packet must not be touched until it is
     * reaped.  A packet t's predicate rejects passes through untouched, in
     * order.  Returns false, submitting nothing, when the queue is full: reap
     * first.
     */
    public boolean submit(GpuTransformerBase t, RawPacket pkt, boolean reverse)
    {
        if (submitted - reaped == ring.length)
            return false;
        boolean skip = t.packetPredicate != null && !t.packetPredicate.test(pkt);
        int i = (int) (submitted % ring.length);
        ring[i] = pkt;
        int rc = SrtpMi355x.queueSubmit(q, reverse, t.tid, pkt, skip, submitted);
        if (rc == SrtpMi355x.EAGAIN)
        {
            ring[i] = null;
            return false;
        }
        SrtpMi355x.check(rc);
        submitted++;
        return true;
    }

    /**
     * Hands the completed packets to sink in submission order: each
     * transformed in place (or moved to a new buffer where RawPacket.append /
     * grow reallocate), or null where SRTPTransformer returns null.  Where the
     * reference throws (a malformed packet) the packet is counted and logged as
     * SinglePacketTransformer does (:134-155) and handed on as null: no caller
     * remains to rethrow to.  wait: block until at least one is done.  Returns
     * the number handed on.
     */
    public int reap(Sink sink, boolean wait)
    {
        if (submitted == reaped)
            return 0;
        int n = SrtpMi355x.check(SrtpMi355x.queueReap(q, ring, status, wait));
        for (int k = 0; k < n; k++)
        {
            int i = (int) (reaped % ring.length);
            RawPacket pkt = ring[i];
            ring[i] = null;
            reaped++;
            int st = status[k];
            if (st == GpuTransformerBase.STATUS_ERR_MALFORMED)
            {
                exceptions++;
                if (exceptions == 1 || exceptions % EXCEPTIONS_TO_LOG == 0)
                    logger.error("Failed to transform RawPacket(s)! (" + exceptions + ")");
            }
            sink.accept(st == GpuTransformerBase.STATUS_OK || st == GpuTransformerBase.STATUS_SKIPPED
                            ? pkt : null);
        }
        return n;
    }

    /** submit, reaping into sink while the queue is full. */
    public void transform(GpuTransformerBase t, RawPacket pkt, boolean reverse, Sink sink)
    {
        while (!submit(t, pkt, reverse))
            reap(sink, true);
    }

    /** Reaps until nothing is in flight. */
    public void drain(Sink sink)
    {
        while (submitted != reaped)
            reap(sink, true);
    }

    public int outstanding()
    {
        return (int) (submitted - reaped);
    }

    /** Waits for the packets in flight (their results are dropped) and frees the queue. */
    public void close()
    {
        SrtpMi355x.queueDestroy(q);
    }
}
